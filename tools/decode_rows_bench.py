"""Decode-step cost of several windows in one step (cbw_decoder_step_rows) vs one window's step, and the
WindowBatcher's whole iteration (per-window scoring + reorder + step) -- GPU time from events, host time from
the wall clock.  usage: python tools/decode_rows_bench.py [model] [steps]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.decoder import DecoderEngine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 48
only = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 3]
beams = 5
dev = torch.device("cuda:0")
cfg = synth.WHISPER_DECODERS[model]
V, D, L, H, F = cfg
sd = synth.synth_whisper_decoder_state_dict(model, seed=0)
dec = DecoderEngine(cfg, sd, dev)
enc = torch.randn((1500, D), device=dev)
prefix = [50258, 50259, 50360, 50364]


def timed(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, (time.perf_counter() - t) * 1e3 / n


# one window, the classic step
dec.start(enc[None], beams)
tok = [50258] * beams
pos = [4]


def one():
    dec.step(tok, pos[0])
    pos[0] += 1


if 0 in only or len(sys.argv) <= 3:
    g, w = timed(one, steps)
    print(f"step (1 window x {beams} beams): {g:.3f} ms GPU-event, {w:.3f} ms wall")
for wins in [x for x in only if x > 0]:
    dec.start_windows(wins, beams)
    for s in range(wins):
        dec.set_window(s, enc)
        dec.prefill_window(s, beams, prefix)
    rows = wins * beams
    toks = torch.full((rows,), 50258, dtype=torch.int32, device=dev)
    inc = torch.ones((rows,), dtype=torch.int32, device=dev)

    def many():
        dec.step_rows(toks)
        dec._posr.add_(inc)

    g, w = timed(many, steps)
    print(f"step_rows ({wins} windows x {beams} beams = {rows} rows): {g:.3f} ms GPU-event, {w:.3f} ms wall, "
          f"{g / wins:.3f} ms per window-step")
