set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_transformer_ops.py tests/test_gpu_defer_wgrad.py tests/test_gpu_lm_head.py -x -q --timeout 120 --timeout-method thread > $O/slab_t.log 2>&1 || { tail -20 $O/slab_t.log; exit 1; }
tail -1 $O/slab_t.log
for m in bert gpt2; do
  for r in 1 2; do
    for arm in on off; do
      if [ $arm = off ]; then export DCP_NO_GRAD_SLAB=1; else unset DCP_NO_GRAD_SLAB; fi
      timeout -k 10 400 python -u bench.py --model $m --steps 20 --warmup 8 > $O/slab_run.log 2>&1 || { tail -5 $O/slab_run.log; exit 1; }
      grep '^{' $O/slab_run.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['label']='$m $arm'; print(json.dumps(d))" >> $O/r5_grad_slab_ab.jsonl
      tail -1 $O/r5_grad_slab_ab.jsonl | cut -c1-120
    done
  done
done
