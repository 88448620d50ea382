"""H2D copy bandwidth on the GPU box: page-locked host -> HBM, one 128 MB copy alone, two on two
streams at once, and one beside a busy kernel stream."""
import time

import torch

MB = 1 << 20


def bw(n_bytes, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return n_bytes * reps / (time.perf_counter() - t) / 1e9


def main():
    n = 128 * MB
    h = [torch.empty(n // 4, dtype=torch.float32).pin_memory() for _ in range(2)]
    d = [torch.empty(n // 4, dtype=torch.float32, device="cuda") for _ in range(2)]
    s = [torch.cuda.Stream() for _ in range(2)]

    def one():
        with torch.cuda.stream(s[0]):
            d[0].copy_(h[0], non_blocking=True)

    def two():
        for i in range(2):
            with torch.cuda.stream(s[i]):
                d[i].copy_(h[i], non_blocking=True)

    print(f"one 128 MB copy: {bw(n, one):.1f} GB/s")
    print(f"two 128 MB copies on two streams: {bw(2 * n, two):.1f} GB/s")
    a = torch.randn(8192, 8192, device="cuda")

    def busy():
        with torch.cuda.stream(s[1]):
            for _ in range(4):
                a.mul_(1.0000001)
        one()

    print(f"one copy beside an elementwise stream: {bw(n, busy):.1f} GB/s")


if __name__ == "__main__":
    main()
