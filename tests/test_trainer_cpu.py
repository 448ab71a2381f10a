"""Trainer CLI end to end on CPU (host backend, 2 ranks): train, eval,
checkpoint, resume with the LR schedule and epoch counter restored."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO)
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-m", "distributed_compute_pytorch_amd.train", "--no-cuda", "--gpus", "2",
                        "--log-every", "2"] + args, capture_output=True, text=True, cwd=tmp_path, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_train_checkpoint_resume(tmp_path):
    ck = str(tmp_path / "ck.pt")
    ev = _run(["--model", "convnet", "--epochs", "1", "--steps-per-epoch", "3", "--checkpoint", ck, "--save-model",
               str(tmp_path / "m.pt")], tmp_path)
    assert any(e["event"] == "eval" for e in ev)
    ev2 = _run(["--model", "convnet", "--epochs", "2", "--steps-per-epoch", "2", "--resume", ck, "--checkpoint", ck,
                "--save-model", str(tmp_path / "m.pt")], tmp_path)
    assert any(e["event"] == "resumed" and e["epoch"] == 0 for e in ev2)
    tr = [e for e in ev2 if e["event"] == "train"]
    assert tr and all(e["epoch"] == 1 for e in tr)
    assert abs(tr[0]["lr"] - 1e-3 * 0.7) < 1e-9
    import torch

    sd = torch.load(str(tmp_path / "m.pt"), weights_only=True)
    assert all(k.startswith("module.") for k in sd)
