"""Calibration of the one-GPU contention emulator (comm_emulate_kernel,
csrc/kernels/multi_tensor.hip): the device time of one emulated 8-rank ring
all-reduce of B bytes at several modelled bus bandwidths, (a) alone on an
idle GPU and (b) while a stream of 256 x 256 GEMMs (one workgroup per CU)
holds the CUs — the emulator is bandwidth-bound only where (a) tracks the
model. One JSON line per (size, busbw, load).

    DCP_SINGLE_RANK_HOP=1 python tools/emu_calib.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCP_SINGLE_RANK_HOP", "1")


def main():
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd._ext import C
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    pg = dcp.distributed.get_default_group()
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    x = torch.randn(8192, 3072, device=dev).to(torch.bfloat16)
    w = torch.randn(3072, 3072, device=dev).to(torch.bfloat16)
    for mb in (4, 16, 50):
        buf = torch.zeros(mb * 2**20 // 4, device=dev)
        comm = pg.comm_for(buf)
        for bw in (150.0, 300.0, 450.0):
            for load in (False, True):
                model_us = 20.0 + 2 * 7 / 8 * buf.numel() * 4 / (bw * 1e3)
                ts = []
                for _ in range(5):
                    if load:
                        with torch.cuda.stream(side):
                            for _ in range(30):
                                C.gemm_pp(x, w)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    cs = torch.cuda.current_stream()
                    s.record(cs)
                    work = comm.emulate_all_reduce(buf, 8, bw, 16, 20.0)
                    work.wait()
                    e.record(cs)
                    torch.cuda.synchronize()
                    ts.append(s.elapsed_time(e) * 1e3)
                ts.sort()
                print(json.dumps({"bucket_mb": mb, "busbw_gbps": bw, "gemm_load": load, "model_us": round(model_us, 1),
                                  "median_us": round(ts[len(ts) // 2], 1), "min_us": round(ts[0], 1)}), flush=True)
    dcp.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
