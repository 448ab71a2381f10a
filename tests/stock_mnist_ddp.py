#!/usr/bin/env python3
"""Stock-PyTorch twin of examples/mnist_ddp.py for the end-to-end parity test
(tests/test_mnist_example_cpu.py): torch.multiprocessing.spawn, the gloo
process group, torch.nn.parallel.DistributedDataParallel, torch.optim.Adadelta
+ StepLR, torch's DistributedSampler with set_epoch — the reference's stack
(main.py:98-134) with the same fixes the example makes (eval on the held-out
split, averaged loss print). Same data (the package's learnable synthetic
MNIST), same seed, same printed lines.

    python tests/stock_mnist_ddp.py --gpus 2 --epochs 2 --lr 1.0 --synthetic-n 1536 --out /tmp/stock.pt
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F
from torch import nn
from torch.nn.parallel import DistributedDataParallel as DDP
from torch.optim.lr_scheduler import StepLR
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class ConvNet(nn.Module):  # the reference architecture, stock modules (main.py:20-45)
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout2d(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)
        self.batchnorm = nn.BatchNorm1d(128)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = F.relu(self.batchnorm(self.fc1(x)))
        x = self.dropout2(x)
        return F.log_softmax(self.fc2(x), dim=1)


def _data(n):
    # the package's dataset module only (data generation is not under test)
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "dcp_data", os.path.join(REPO, "distributed_compute_pytorch_amd", "utils", "data.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.SyntheticDataset(n, seed=0), mod.SyntheticDataset(n // 6, seed=1)


def proc(rank, world_size, opt):
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    torch.manual_seed(0)
    train_ds, test_ds = _data(opt.synthetic_n)
    train_sampler = DistributedSampler(train_ds, num_replicas=world_size, rank=rank)
    test_sampler = DistributedSampler(test_ds, num_replicas=world_size, rank=rank, shuffle=False)
    train_loader = DataLoader(train_ds, batch_size=opt.batch_size, sampler=train_sampler)
    test_loader = DataLoader(test_ds, batch_size=opt.batch_size, sampler=test_sampler)
    model = DDP(ConvNet())
    optimizer = torch.optim.Adadelta(model.parameters(), lr=opt.lr)
    scheduler = StepLR(optimizer, step_size=1, gamma=opt.gamma)
    for epoch in range(opt.epochs):
        t0 = time.time()
        train_sampler.set_epoch(epoch)
        model.train()
        for b, (img, label) in enumerate(train_loader):
            optimizer.zero_grad()
            loss = F.nll_loss(model(img), label)
            loss.backward()
            optimizer.step()
            if b % 10 == 0:
                t = loss.detach().clone()
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                t /= world_size
                if rank == 0:
                    print(f"epoch: {epoch} [{b}/{len(train_loader)} ({100. * b / len(train_loader):.0f}%)]\t "
                          f"Loss:{t.item():.6f}", flush=True)
        model.eval()
        s = torch.zeros(()); c = torch.zeros((), dtype=torch.long); n = torch.zeros((), dtype=torch.long)
        with torch.no_grad():
            for img, label in test_loader:
                out = model(img)
                s += F.nll_loss(out, label, reduction="sum")
                c += out.argmax(dim=1).eq(label).sum()
                n += label.numel()
        for t in (s, c, n):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if rank == 0:
            print(f"\nTest set: Average loss: {s.item() / max(1, n.item()):.4f}, Accuracy: {c.item()}/{n.item()} "
                  f"({100. * c.item() / max(1, n.item()):.0f}%)\n", flush=True)
        scheduler.step()
        if rank == 0:
            print(f"time to complete this epoch: {time.time() - t0} seconds", flush=True)
    dist.barrier()
    if rank == 0:
        torch.save(model.state_dict(), opt.out)
    dist.barrier()
    dist.destroy_process_group()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch_size", type=int, default=128)
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--epochs", type=int, default=20)
    p.add_argument("--gamma", default=0.7, type=float)
    p.add_argument("--gpus", default=2, type=int)
    p.add_argument("--synthetic-n", type=int, default=60000)
    p.add_argument("--out", default="stock_mnist.pt")
    opt = p.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    mp.spawn(proc, args=(opt.gpus, opt), nprocs=opt.gpus, join=True)


if __name__ == "__main__":
    sys.exit(main())
