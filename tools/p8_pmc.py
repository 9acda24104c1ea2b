"""One plain-GEMM launch shape (1x1, M 65536, K 2048, N 2048) on conv_igemm_p8, repeated: a target for
rocprofv3 --pmc (LDS bank conflicts, wait cycles)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import _lib  # noqa: E402

lib = _lib.load()
d = torch.device("cuda:0")
N, H, W, Cin, Cout, k = [int(v) for v in os.environ.get("P8_SHAPE", "1,1,65536,2048,2048,1").split(",")]
p = k // 2
x = torch.randn((N, H, W, Cin), device=d).to(torch.bfloat16)
w = (torch.randn((Cout, k, k, Cin), device=d) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
b = torch.randn(Cout, device=d)
y = torch.empty((N, H, W, Cout), device=d, dtype=torch.bfloat16)
for _ in range(5):
    _lib.check(lib.cbw_conv2d(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(), N, H, W, Cin, Cout, k, k,
                              1, 1, p, p, 1, _lib.stream_handle()), "conv")
torch.cuda.synchronize()
print("ok")
