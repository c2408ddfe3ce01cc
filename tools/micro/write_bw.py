"""Achievable HBM write bandwidth on the box (the trace-back's floor): fill_ of a 1.66 GB
buffer (the trace-back's history bytes at 1M x 100) and of 101 separate 16 MB columns, timed
with events; and a copy (read + write) for comparison. python tools/micro/write_bw.py"""
import torch

dev = torch.device("cuda:0")


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


n = 1_000_000 * 101 * 2
big = torch.empty(n, dtype=torch.float64, device=dev)
cols = [torch.empty(2_000_000, dtype=torch.float64, device=dev) for _ in range(101)]
src = torch.empty(n, dtype=torch.float64, device=dev).fill_(1.0)
b = n * 8
t = timed(lambda: big.fill_(1.0))
print(f"fill one buffer {b / 1e9:.2f} GB: {t * 1e6:.1f} us = {b / t / 1e12:.2f} TB/s")
t = timed(lambda: [c.fill_(2.0) for c in cols])
print(f"fill 101 columns of 16 MB: {t * 1e6:.1f} us = {b / t / 1e12:.2f} TB/s")
t = timed(lambda: big.copy_(src))
print(f"copy (read + write) {b / 1e9:.2f} GB: {t * 1e6:.1f} us = {2 * b / t / 1e12:.2f} TB/s moved")
