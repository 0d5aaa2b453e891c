"""Practical HBM bandwidth on this box (context for the roofline fractions): a 4 GiB
device copy (read + write), a read-only reduction and a write-only fill, timed with HIP events."""
import json
import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 30  # int32 elements: 4 GiB
    x = torch.ones(n, dtype=torch.int32, device=dev)
    y = torch.empty_like(x)
    out = {}
    t = timed(lambda: y.copy_(x))
    out["copy_TBps"] = 2 * 4 * n / t / 1e12
    xf = x.view(torch.float32)
    t = timed(lambda: xf.sum())
    out["read_sum_f32_TBps"] = 4 * n / t / 1e12
    t = timed(lambda: torch.add(x, 1, out=y))
    out["add_TBps"] = 2 * 4 * n / t / 1e12
    t = timed(lambda: y.fill_(7))
    out["write_fill_TBps"] = 4 * n / t / 1e12
    out["bytes_per_op_GiB"] = 4
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
