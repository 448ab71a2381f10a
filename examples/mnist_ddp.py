#!/usr/bin/env python3
"""The reference training script (main.py) on this framework.

Same CLI flags and defaults as the reference (main.py:138-145), same loop
structure (train: main.py:55-68, test: main.py:70-95, proc: main.py:98-134),
with the quirks SURVEY App. A marks as "fix" fixed: device follows
availability (A2/A3), DDP always wraps (A4), set_epoch each epoch (A6), eval
on the held-out split (A7), rank-0-only save behind a barrier (A10),
env-overridable rendezvous (A11), on-device metric accumulation (A9).
`--parity` restores the reference's logging of summed (not averaged) losses.

    python examples/mnist_ddp.py --gpus 2 --epochs 1            # GPUs: RCCL
    python examples/mnist_ddp.py --no-cuda --gpus 2 --epochs 1  # CPU: host backend
Data: MNIST IDX files under --data if present, otherwise MNIST-shaped synthetic.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_compute_pytorch_amd as dcp  # noqa: E402
from distributed_compute_pytorch_amd.models import ConvNet  # noqa: E402
from distributed_compute_pytorch_amd.utils import DistributedSampler, MNISTIdx, SyntheticDataset  # noqa: E402


def train(opt, model, device, loader, optimizer, epoch, rank):
    model.train()
    for b, (img, label) in enumerate(loader):
        img, label = img.to(device, non_blocking=True), label.to(device, non_blocking=True)
        optimizer.zero_grad()
        loss = F.nll_loss(model(img), label)
        loss.backward()
        optimizer.step()
        if b % 10 == 0:
            t = loss.detach().clone()
            dcp.distributed.all_reduce(t, op=dcp.distributed.ReduceOp.SUM)
            if not opt.parity:
                t /= dcp.distributed.get_world_size()
            if rank == 0:
                print(f"epoch: {epoch} [{b}/{len(loader)} ({100. * b / len(loader):.0f}%)]\t Loss:{t.item():.6f}")


def test(opt, model, device, loader, rank):
    model.eval()
    loss_sum = torch.zeros((), device=device)
    correct = torch.zeros((), device=device, dtype=torch.long)
    n = torch.zeros((), device=device, dtype=torch.long)
    with torch.no_grad():
        for img, label in loader:
            img, label = img.to(device), label.to(device)
            out = model(img)
            loss_sum += F.nll_loss(out, label, reduction="sum")
            correct += out.argmax(dim=1).eq(label).sum()
            n += label.numel()
    for t in (loss_sum, correct, n):
        dcp.distributed.all_reduce(t, op=dcp.distributed.ReduceOp.SUM)
    if rank == 0:
        avg = loss_sum.item() if opt.parity else loss_sum.item() / max(1, n.item())
        print(f"\nTest set: Average loss: {avg:.4f}, Accuracy: {correct.item()}/{n.item()} "
              f"({100. * correct.item() / max(1, n.item()):.0f}%)\n")


def proc(rank, world_size, opt, use_cuda):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    dcp.distributed.init_process_group("rccl" if use_cuda else "gloo", rank=rank, world_size=world_size)
    device = torch.device("cuda", rank) if use_cuda else torch.device("cpu")
    torch.manual_seed(0)
    try:
        train_ds, test_ds = MNISTIdx(opt.data, True), MNISTIdx(opt.data, False)
    except FileNotFoundError:
        train_ds, test_ds = SyntheticDataset(opt.synthetic_n, seed=0), SyntheticDataset(opt.synthetic_n // 6, seed=1)
    train_sampler = DistributedSampler(train_ds, num_replicas=world_size, rank=rank)
    test_sampler = DistributedSampler(test_ds, num_replicas=world_size, rank=rank, shuffle=False)
    train_loader = DataLoader(train_ds, batch_size=opt.batch_size, sampler=train_sampler, pin_memory=use_cuda)
    test_loader = DataLoader(test_ds, batch_size=opt.batch_size, sampler=test_sampler, pin_memory=use_cuda)
    # fused=True on a GPU: the fp32-MFMA feature extractor (convnet.hip), fused
    # BN1d + ReLU, Philox dropout and log-softmax kernels; identical parameters
    # and state_dict keys (models/convnet.py), so checkpoints load either way
    model = dcp.parallel.DistributedDataParallel(ConvNet(fused=use_cuda).to(device),
                                                 device_ids=[rank] if use_cuda else None)
    optimizer = dcp.optim.Adadelta(model.parameters(), lr=opt.lr)
    scheduler = dcp.optim.StepLR(optimizer, step_size=1, gamma=opt.gamma)
    for epoch in range(opt.epochs):
        t0 = time.time()
        train_sampler.set_epoch(epoch)
        train(opt, model, device, train_loader, optimizer, epoch, rank)
        test(opt, model, device, test_loader, rank)
        scheduler.step()
        if rank == 0:
            print(f"time to complete this epoch: {time.time() - t0} seconds")
    dcp.utils.save_model(model, opt.out)
    dcp.distributed.destroy_process_group()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch_size", type=int, default=128, help="batch size of train and test")
    p.add_argument("--lr", type=float, default=0.001, help="LR of optimizer")
    p.add_argument("--epochs", type=int, default=20, help="#of epochs")
    p.add_argument("--no-cuda", action="store_true", default=False, help="disables GPUs")
    p.add_argument("--gamma", default=0.7, type=float, help="gamma value for lr update")
    p.add_argument("--gpus", default=4, type=int, help="# of processes (GPUs)")
    p.add_argument("--data", default="./data", help="directory holding MNIST IDX files")
    p.add_argument("--synthetic-n", type=int, default=60000)
    p.add_argument("--out", default="mnist.pt")
    p.add_argument("--parity", action="store_true", help="reference logging (summed losses)")
    opt = p.parse_args()
    use_cuda = not opt.no_cuda and torch.cuda.is_available()
    world_size = opt.gpus
    if use_cuda and world_size > torch.cuda.device_count():
        raise SystemExit(f"--gpus {world_size} but only {torch.cuda.device_count()} GPUs visible")
    os.environ.setdefault("MASTER_PORT", str(dcp.distributed.launch.free_port()))
    dcp.distributed.launch.spawn(proc, args=(world_size, opt, use_cuda), nprocs=world_size, join=True)


if __name__ == "__main__":
    main()
