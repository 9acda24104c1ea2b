"""Ceiling probe: hipBLASLt (torch.matmul, bf16) and MIOpen (torch conv2d, channels_last bf16) on the
GEMM / conv shapes of the LEF ResNet-50 convs at a chunk of 500 pairs, for comparison with the
libcbw conv kernels (tools/layer_bench.py).  Prints TFLOP/s per shape."""
import torch
import torch.nn.functional as F

d = torch.device("cuda:0")
P = 500
# (name, H, W, Cin, Cout, k, stride)
shapes = [
    ("s1.mid", 19, 188, 64, 64, 3, 1),
    ("s2.reduce", 10, 94, 512, 128, 1, 1),
    ("s2.mid", 10, 94, 128, 128, 3, 1),
    ("s2.expand", 10, 94, 128, 512, 1, 1),
    ("s3.reduce", 5, 47, 1024, 256, 1, 1),
    ("s3.mid", 5, 47, 256, 256, 3, 1),
    ("s3.expand", 5, 47, 256, 1024, 1, 1),
    ("s4.reduce", 3, 24, 2048, 512, 1, 1),
    ("s4.mid", 3, 24, 512, 512, 3, 1),
    ("s4.expand", 3, 24, 512, 2048, 1, 1),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for name, H, W, cin, cout, k, s in shapes:
    M = P * H * W
    K = cin * k * k
    fl = 2.0 * M * cout * K
    a = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    b = torch.randn(K, cout, device=d, dtype=torch.bfloat16)
    t = timeit(lambda: a @ b)
    x = torch.randn(P, cin, H, W, device=d, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, k, k, device=d, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    try:
        tc = timeit(lambda: F.conv2d(x, w, padding=k // 2))
        conv = f"{fl / tc / 1e12:7.1f} TFLOP/s ({tc * 1e6:7.1f} us)"
    except Exception as e:  # noqa: BLE001
        conv = f"conv failed: {e}"
    print(f"{name:10s} M={M:7d} N={cout:5d} K={K:5d}: hipBLASLt {fl / t / 1e12:7.1f} TFLOP/s ({t * 1e6:7.1f} us)"
          f" | MIOpen {conv}", flush=True)
    del a, b, x, w
    torch.cuda.empty_cache()
