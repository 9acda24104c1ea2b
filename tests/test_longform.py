"""Long-form generation (PBAWhisper.generate > 30 s, src/model/pba_whisper.py:343-475) — CPU.

Golden: tests/golden/longform_micro.npz — transformers 5.15 WhisperForConditionalGeneration.generate on
the micro model (seeded weights), greedy, return_timestamps=True, 70 s of audio, with every window's
seek, decoder prompt and post-processed tokens recorded (make_golden.py longform).  The reference pins
transformers 4.37.2 (absent); the functions restated here are the same in both for one audio at
temperature 0 (DESIGN.md §9 lists the one difference: the segment end time of a window without a
timestamp pair, which 4.37 computes as time_offset + seek_num_frames * 0.02).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

TB, NO_TS, EOS, SOP = 50364, 50363, 50257, 50361


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "longform_micro.npz"))


def rows(a):
    return [[int(t) for t in r if t >= 0] for r in a]


def test_seek_loop_replays_hf(g):
    """cbw.timestamps.longform_generate driven by HF's own window outputs reproduces HF's prompts, seeks,
    segments and final sequence (the host logic: prompt prefix, window post-processing, segment split)."""
    from cbw.timestamps import longform_generate
    prefixes, windows = rows(g["prefix"]), rows(g["window"])
    T = g["features"].shape[-1]
    calls = {"seek": [], "prefix": []}

    def window(seek, n):
        calls["seek"].append((seek, n))
        return len(calls["seek"]) - 1

    def decode(w, prefix, begin):
        calls["prefix"].append(list(prefix))
        assert begin == len(prefix)
        return list(prefix) + windows[w] + [EOS]

    seq, segs = longform_generate(T, window, lambda w: [], decode, [50258, 50259, 50359], SOP, EOS, TB, False)
    assert [s for s, _ in calls["seek"]] == g["seek"].tolist()
    assert [n for _, n in calls["seek"]] == g["nframes"].tolist()
    assert calls["prefix"] == prefixes
    # transformers 5.x keeps the second timestamp of a window's closing pair in that window's last segment
    # ("slices[-1] += 1"); 4.37.2, the pinned version restated here, leaves it out (the seek is the same)
    want = [t[:-1] if len(t) >= 2 and t[-1] >= TB and t[-2] >= TB else t for t in rows(g["seg_tokens"])]
    assert [s["tokens"] for s in segs] == want
    assert seq == [t for w in want for t in w]
    assert len(g["sequence"]) - len(seq) == sum(len(a) - len(b) for a, b in zip(rows(g["seg_tokens"]), want))
    np.testing.assert_allclose([s["start"] for s in segs], g["seg_start"], atol=1e-9)
    paired = [i for i, s in enumerate(segs) if s["tokens"][-1] >= TB]
    np.testing.assert_allclose([segs[i]["end"] for i in paired], g["seg_end"][paired], atol=1e-9)


def test_retrieve_segment_and_strip_cases():
    from cbw.timestamps import prompt_prefix, retrieve_segment, strip_window
    # two closed segments, then an unfinished one: seek to the last closed end timestamp (x2 frames)
    seq = [TB + 0, 11, TB + 5, TB + 5, 12, TB + 9, TB + 9, 13, 14]
    segs, off = retrieve_segment(seq, 10.0, TB, 3000)
    assert [s["tokens"] for s in segs] == [[TB, 11, TB + 5], [TB + 5, 12, TB + 9]] and off == 9 * 2
    assert segs[1]["start"] == pytest.approx(10.1) and segs[1]["end"] == pytest.approx(10.18)
    # single timestamp ending: the remainder is a segment, seek the whole window
    segs, off = retrieve_segment([TB, 11, TB + 5, TB + 5, 12, TB + 7], 0.0, TB, 2500)
    assert [s["tokens"] for s in segs] == [[TB, 11, TB + 5], [TB + 5, 12, TB + 7]] and off == 2500
    # no pair: one segment, its end from the last timestamp, seek the window
    segs, off = retrieve_segment([TB + 3, 11, 12, TB + 40], 5.0, TB, 3000)
    assert len(segs) == 1 and segs[0]["end"] == pytest.approx(5.8) and off == 3000
    segs, off = retrieve_segment([11, 12], 5.0, TB, 3000)   # no timestamps at all (4.37: frames * precision)
    assert segs[0]["end"] == pytest.approx(5.0 + 3000 * 0.02) and off == 3000
    assert strip_window([5, 6, EOS], EOS, EOS, is_final=False) == [5, 6]
    assert strip_window([5, 6, EOS], EOS, EOS, is_final=True) == [5, 6]
    assert strip_window([5, 6], EOS, EOS, is_final=False) == [5, 6]
    # prompt: keywords (3/4 of the half context when conditioning), previous tokens, init tokens
    init = [50258, 50259, 50359]
    assert prompt_prefix([], [], init, SOP, True) == init
    assert prompt_prefix([7, 8], [], init, SOP, False) == [SOP, 7, 8] + init
    p = prompt_prefix(list(range(300)), list(range(1000, 1100)), init, SOP, True)
    assert p[0] == SOP and p[1:167] == list(range(300))[-166:] and p[167:-3] == list(range(1100 - 56, 1100))


def test_timestamp_mask_matches_hf_processor():
    """oracle.decoder.timestamp_mask == transformers' WhisperTimeStampLogitsProcessor on random rows (the
    installed 5.15 class; its __call__ is the 4.37.2 one)."""
    import torch
    from transformers import GenerationConfig
    from transformers.generation.logits_process import WhisperTimeStampLogitsProcessor
    from oracle.decoder import timestamp_mask
    V = 51865
    rng = np.random.default_rng(0)
    gc = GenerationConfig(eos_token_id=EOS, no_timestamps_token_id=NO_TS, max_initial_timestamp_index=50)
    begin = 4
    cases = [[], [TB + 3], [TB + 3, 17], [TB + 3, 17, TB + 9], [TB + 3, 17, TB + 9, TB + 9], [11, 12],
             [TB, TB], [TB + 2, 5, 6, TB + 2]]
    for sampled in cases:
        for scale in (1.0, 6.0):
            x = rng.standard_normal(V) * scale
            x[TB:] -= rng.uniform(0, 6)             # vary the timestamp mass
            proc = WhisperTimeStampLogitsProcessor(gc, begin_index=begin)
            ids = torch.tensor([[50258, 50259, 50359, 50364][:begin] + sampled])
            ref = proc(ids, torch.from_numpy(x[None]).float())[0].numpy()
            got = timestamp_mask(x, sampled, TB, NO_TS, EOS, 50)
            np.testing.assert_array_equal(np.isinf(ref), np.isinf(got), err_msg=str(sampled))


def test_oracle_greedy_window_matches_hf(g):
    """The oracle decoder under the oracle timestamp rules, greedy, reproduces the first tokens HF decoded
    in window 1 (bounded: the oracle re-runs the whole prefix per step)."""
    import oracle.encoder as oenc
    from cbw import synth
    from cbw.generate import greedy
    from oracle.decoder import oracle_step_fn
    enc_sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    dec_sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    feats = g["features"][:, :3000].astype(np.float32)
    enc = oenc.encoder_hidden_states(enc_sd, feats, synth.WHISPER_CONFIGS["micro"][3])[-1]
    prefix = rows(g["prefix"])[0]
    V = synth.WHISPER_DECODERS["micro"][0]
    base = np.zeros(V)
    base[[1, 2, 7]] = -np.inf
    begin_b = base.copy()
    begin_b[[220, EOS]] = -np.inf
    bias_at = lambda pos: begin_b if pos == len(prefix) else base   # noqa: E731
    n = 24
    step = oracle_step_fn(dec_sd, enc, synth.WHISPER_DECODERS["micro"][3], 4, bias_at, (TB, NO_TS, EOS, 50), len(prefix))
    out = greedy(step, prefix, EOS, len(prefix) + n)
    assert out[len(prefix):] == rows(g["window"])[0][:n]


@pytest.fixture(scope="module")
def gb():
    return np.load(os.path.join(GOLDEN, "longform_batched_micro.npz"))


def test_batched_seek_loop_replays_hf(gb):
    """cbw.timestamps.longform_generate_batched (pba_whisper.py:351-475 with batch_size > 1) driven by HF's own window
    outputs (tests/golden/longform_batched_micro.npz: transformers 5.15 batched long-form generate, three audios of
    70 / 45 / 95 s, padded features + attention_mask, greedy, timestamps, no conditioning) reproduces HF's batch
    reduction (which audios each iteration decodes, in order), every audio's seeks and window lengths, the decoder
    inputs, and every audio's segments and sequence (the 4.37.2 closing-pair rule, as test_seek_loop_replays_hf)."""
    from cbw.timestamps import longform_generate_batched
    max_frames = gb["attention_mask"].sum(-1).tolist()
    maps = [[b for b in r if b >= 0] for r in gb["call_map"].tolist()]
    seeks = [[s for s in r if s >= 0] for r in gb["call_seek"].tolist()]
    nfr = [[s for s in r if s >= 0] for r in gb["call_nframes"].tolist()]
    windows = rows(gb["call_window"])
    calls = []

    def window(b, seek, n):
        calls[-1].append((b, seek, n)) if calls and len(calls[-1]) < len(maps[len(calls) - 1]) else calls.append([(b, seek, n)])
        return (len(calls) - 1, b)

    taken = [0]

    def decode(segs, prefixes, begin):
        c = segs[0][0]
        got = [list(p) for p in gb["call_prefix"][c][:len(segs)].tolist()]
        assert [list(p) for p in prefixes] == got and all(len(p) == begin for p in prefixes)
        out = []
        for _ in segs:
            out.append(list(prefixes[0]) + windows[taken[0]] + [EOS])
            taken[0] += 1
        return out

    seqs, segs = longform_generate_batched(max_frames, window, lambda s: [[] for _ in s], decode, [50258, 50259, 50359],
                                           SOP, EOS, TB, False)
    assert [[b for b, _, _ in c] for c in calls] == maps
    assert [[s for _, s, _ in c] for c in calls] == seeks
    assert [[n for _, _, n in c] for c in calls] == nfr
    assert taken[0] == len(windows)
    for b in range(3):
        want = [t[:-1] if len(t) >= 2 and t[-1] >= TB and t[-2] >= TB else t for t in rows(gb[f"seg_tokens_{b}"])]
        assert [s["tokens"] for s in segs[b]] == want, f"audio {b}: segments differ"
        assert seqs[b] == [t for w in want for t in w]
        np.testing.assert_allclose([s["start"] for s in segs[b]], gb[f"seg_start_{b}"], atol=1e-9)


def test_batched_prompt_prefixes_follow_prepare_decoder_input_ids():
    """batched_prompt_prefixes restates pba_whisper.py:478-548 with 4.37.2's _pad_to_max_length: keyword lists left-
    padded to the longest (cut to 166 tokens when any audio conditions, 222 otherwise), the previous tokens left-padded
    and cut to 223 - keyword width - 1 (only when audio 0 of the batch has segments), [<|startofprev|>] + both + init;
    nothing to prompt -> the init tokens; one audio -> prompt_prefix's layout."""
    from cbw.timestamps import batched_prompt_prefixes, prompt_prefix
    init, PAD = [50258, 50259, 50359], EOS
    kw = [[11, 12], [13], []]
    prev = [[21, 22, 23], None, [31]]
    out = batched_prompt_prefixes(kw, prev, init, SOP, PAD, True, True)
    assert out == [[SOP, 11, 12, 21, 22, 23] + init, [SOP, PAD, 13, PAD, PAD, PAD] + init,
                   [SOP, PAD, PAD, PAD, PAD, 31] + init]
    # audio 0 without segments: no previous tokens for anyone (pba_whisper.py:520 tests current_segments[0])
    assert batched_prompt_prefixes(kw, prev, init, SOP, PAD, True, False) == \
        [[SOP, 11, 12] + init, [SOP, PAD, 13] + init, [SOP, PAD, PAD] + init]
    assert batched_prompt_prefixes([[], []], [None, None], init, SOP, PAD, False, False) == [init, init]
    long_kw = list(range(1000, 1300))
    a = batched_prompt_prefixes([long_kw, [5]], [list(range(2000, 2100)), [7]], init, SOP, PAD, True, True)
    assert a[0][1:167] == long_kw[-166:] and a[1][1:167] == [PAD] * 165 + [5]
    assert a[0][167:-3] == list(range(2000, 2100))[-56:] and len(a[0]) == len(a[1]) == 1 + 166 + 56 + 3
    b = batched_prompt_prefixes([long_kw, [5]], [None, None], init, SOP, PAD, False, False)
    assert b[0][1:-3] == long_kw[-222:]
    for k_, p_, c_ in (([11, 12], [21, 22], True), ([11], [], True), ([], [21], True), ([11, 12], [21], False)):
        one = batched_prompt_prefixes([k_], [p_ if c_ else None], init, SOP, PAD, c_, c_ and len(p_) > 0)
        assert one == [prompt_prefix(k_, p_, init, SOP, c_)]
