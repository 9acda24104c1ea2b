"""conv_igemm_p8 vs conv_igemm_big2 on plain GEMM shapes (1x1 convs, random bf16 data) and on the ResNet 3x3
shapes: TFLOP/s per kernel, best of REPS launches, modes interleaved (CBW_CONV_P8=0/1; P8C_VAR / P8C_MODES name
another knob and its modes, e.g. P8C_VAR=CBW_P8_DEEP)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import _lib  # noqa: E402

lib = _lib.load()
d = torch.device("cuda:0")
REPS = 10
VAR = os.environ.get("P8C_VAR", "CBW_CONV_P8")
MODES = os.environ.get("P8C_MODES", "0,1").split(",")
shapes = [  # N, H, W, Cin, Cout, k, s
    (1, 1, 65536, 2048, 2048, 1, 1), (1, 1, 65536, 4096, 1024, 1, 1), (1, 1, 131072, 1024, 1024, 1, 1),
    (625, 5, 47, 256, 256, 3, 1), (625, 3, 24, 512, 512, 3, 1), (625, 5, 47, 1024, 256, 1, 1),
    (625, 10, 94, 256, 256, 3, 2), (625, 3, 24, 2048, 512, 1, 1), (625, 3, 24, 512, 2048, 1, 1)]
for (N, H, W, Cin, Cout, k, s) in shapes:
    x = torch.randn((N, H, W, Cin), device=d).to(torch.bfloat16)
    w = (torch.randn((Cout, k, k, Cin), device=d) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=d)
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = torch.empty((N, Ho, Wo, Cout), device=d, dtype=torch.bfloat16)
    f = 2.0 * N * Ho * Wo * Cout * Cin * k * k
    best = {}
    for rnd in range(3):
        for mode in MODES if rnd % 2 == 0 else MODES[::-1]:
            os.environ[VAR] = mode
            run = lambda: lib.cbw_conv2d(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(), N, H, W, Cin,  # noqa: E731
                                         Cout, k, k, s, s, p, p, 1, _lib.stream_handle())
            _lib.check(run(), "conv")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                run()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / REPS * 1e-3
            best[mode] = min(best.get(mode, 1e9), t)
    rates = "  ".join(f"{VAR}={m} {f / best[m] / 1e12:7.1f}" for m in MODES)
    print(f"{N}x{H}x{W} {Cin}->{Cout} k{k}: {rates} TFLOP/s", flush=True)
