"""Achievable HBM write / copy bandwidth on this device (torch fill_ / copy_), for
judging the bz_i8 epilogue."""
import torch
n = 1 << 28  # 2 GiB of fp64
x = torch.empty(n, dtype=torch.float64, device="cuda")
xl = torch.empty(n * 4, dtype=torch.float64, device="cuda")  # 8 GiB: the bench's B z output per step
y = torch.empty(n // 2, dtype=torch.float64, device="cuda")
z = torch.empty(n // 2, dtype=torch.float64, device="cuda")
for name, fn, nbytes in [("fill_2GiB", lambda: x.fill_(1.0), 8 * n),
                         ("fill_8GiB", lambda: xl.fill_(1.0), 32 * n),
                         ("copy_1GiB", lambda: y.copy_(z), 8 * n)]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name}: {ms:.3f} ms, {nbytes / ms * 1e-6:.0f} GB/s")
