#!/usr/bin/env python3
"""HBM calibration on this GPU: streaming copy (read+write), read-only and write-only rates
with torch kernels on buffers far larger than the 256 MiB Infinity Cache.  The copy rate is
the practical ceiling for a kernel that reads and writes equal byte counts (pulse
compression, MTD)."""
import torch


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


def main():
    n = 1 << 28   # 1 GiB of fp32
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    t = timeit(lambda: y.copy_(x))
    print("copy        %7.1f GB/s (read+write bytes)" % (2 * n * 4 / t / 1e9))
    t = timeit(lambda: x.sum())
    print("read (sum)  %7.1f GB/s" % (n * 4 / t / 1e9))
    t = timeit(lambda: y.fill_(1.0))
    print("write(fill) %7.1f GB/s" % (n * 4 / t / 1e9))
    z = torch.empty(n // 2, dtype=torch.complex64, device="cuda")
    xc = torch.view_as_complex(x.view(-1, 2))
    t = timeit(lambda: torch.mul(xc, 2.0, out=z))
    print("cplx scale  %7.1f GB/s (read+write bytes)" % (2 * n * 4 / t / 1e9))


if __name__ == "__main__":
    main()
