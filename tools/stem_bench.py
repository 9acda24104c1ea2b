"""Time the fused stem + max-pool (cbw_stem_pool) on one LEF scoring chunk ([P, 75, 750, 4] NHWC4 maps -> [P, 19, 188,
64]) with hipEvents, and print a digest of the output so two builds (CBW_LIB=...) can be checked bit-identical.
usage: STEM_PAIRS=625 python tools/stem_bench.py"""
import ctypes
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import _lib  # noqa: E402

P = int(os.environ.get("STEM_PAIRS", "625"))
REPS = int(os.environ.get("STEM_REPS", "20"))
_lib.load()
# cbw_stem_pool is internal (csrc/cbw_kernels.h, C++ linkage): bound here by its mangled name
fn = getattr(ctypes.CDLL(_lib.LIB_PATH), "_Z13cbw_stem_poolPKtS0_PKfPtiiiiiiiP12ihipStream_t")
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 7 + [ctypes.c_void_p]
d = torch.device("cuda:0")
g = torch.Generator(device=d).manual_seed(0)
H, W, Hs, Ws, Hp, Wp = 75, 750, 38, 375, 19, 188
x = torch.rand((P, H, W, 4), device=d, generator=g) * 2 - 1
x[..., 3] = 0
x = x.to(torch.bfloat16)
w = (torch.randn((64, 7, 8, 4), device=d, generator=g) / 12).to(torch.bfloat16)
w[:, :, 7, :] = 0
w[:, :, :, 3] = 0
b = torch.randn(64, device=d, generator=g) * 0.1
y = torch.empty((P, Hp, Wp, 64), device=d, dtype=torch.bfloat16)
st = _lib.stream_handle()


def run():
    rc = fn(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), P, H, W, Hs, Ws, Hp, Wp, st)
    if rc:
        raise RuntimeError(f"cbw_stem_pool: hip error {rc}")


for _ in range(3):
    run()
torch.cuda.synchronize()
best = 1e9
for rnd in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        run()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) * 1e3 / REPS)
digest = hashlib.sha256(y.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
flops = 2.0 * P * Hs * Ws * 64 * 147
byt = P * (H * W * 8 + Hp * Wp * 128)
print(f"stem_pool P={P} {best:.1f} us  {flops / best / 1e6:.0f} TF/s useful  {byt / best / 1e6:.2f} TB/s  "
      f"lib={os.path.basename(_lib.LIB_PATH)} digest={digest}", flush=True)
