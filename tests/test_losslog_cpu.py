"""train._LossLog: loss records are written when their device copies have
landed, in step order, never ahead of an earlier incomplete one; a flush at
the epoch end writes the rest (fake events stand in for HIP events here; the
GPU path is covered by test_gpu_train_graph.py)."""
import torch

from distributed_compute_pytorch_amd.train import _LossLog


class _Log:
    def __init__(self):
        self.rows = []

    def log(self, **kw):
        self.rows.append(kw)


class _Ev:
    def __init__(self, done):
        self.done = done

    def query(self):
        return self.done

    def synchronize(self):
        self.done = True


def _fields(step):
    return dict(epoch=0, step=step, steps=4, lr=1e-3)


def test_poll_keeps_step_order_and_flush_writes_rest():
    log = _Log()
    ll = _LossLog(log)
    evs = [_Ev(True), _Ev(False), _Ev(True)]
    for i, ev in enumerate(evs):
        ll.q.append((torch.tensor(float(i)), ev, _fields(i)))
    ll.poll()
    assert [r["step"] for r in log.rows] == [0]  # step 2 is ready but waits behind step 1
    evs[1].done = True
    ll.poll()
    assert [r["step"] for r in log.rows] == [0, 1, 2]
    ll.q.append((torch.tensor(3.0), _Ev(False), _fields(3)))
    ll.poll(wait=True)
    assert [r["step"] for r in log.rows] == [0, 1, 2, 3] and log.rows[-1]["loss"] == 3.0
    assert list(log.rows[0]) == ["event", "epoch", "step", "steps", "loss", "lr"]


def test_cpu_tensor_logged_immediately():
    log = _Log()
    _LossLog(log).push(torch.tensor(1.25), **_fields(0))
    assert log.rows == [dict(event="train", epoch=0, step=0, steps=4, loss=1.25, lr=1e-3)]
