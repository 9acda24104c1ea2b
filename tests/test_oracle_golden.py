"""Pin the numpy oracle against golden vectors produced by the reference's own
modules (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from cbw import synth
import oracle.kws as okws
from golden_cases import KWS_CASES, THRESHOLDS


@pytest.mark.parametrize("name", list(KWS_CASES))
def test_kws_oracle_matches_reference(name, golden_dir):
    hp, bk = KWS_CASES[name]
    g = np.load(os.path.join(golden_dir, f"kws_{name}.npz"))
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
    km, um = b["kwd_mask"], b["utt_mask"]
    logits, feats = okws.kws_forward(sd, hp, b["kwd"], b["utt"], km, um)
    assert tuple(feats.shape) == tuple(g["feat_shape"])
    np.testing.assert_allclose(feats[:, :, ::7, ::11], g["feat_sub"], atol=2e-5)
    np.testing.assert_allclose(feats.astype(np.float64).sum(axis=(2, 3)), g["feat_sum"], rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(logits, g["logits"], rtol=2e-4, atol=2e-4)
    probs, _ = okws.decide(logits, b["ghost_mask"], 0.5)
    np.testing.assert_allclose(probs, g["probs"], atol=1e-4)
    for t in THRESHOLDS:
        _, idx = okws.decide(logits, b["ghost_mask"], t)
        np.testing.assert_array_equal(idx, g[f"idx_{t}"])
    np.testing.assert_array_equal(okws.spot_argmax(logits), g["argmax_idx"])
    if "feat_full_k0" in g:
        np.testing.assert_allclose(feats[:1], g["feat_full_k0"], atol=2e-5)


@pytest.mark.parametrize("n_mel", [80, 128])
def test_mel_oracle_matches_hf(n_mel, golden_dir):
    from oracle.mel import log_mel
    g = np.load(os.path.join(golden_dir, f"mel_{n_mel}.npz"))
    np.testing.assert_allclose(log_mel(synth.synth_clip(0), n_mel), g["noise_sines"], atol=2e-4)
    sil = log_mel(np.zeros(480000, np.float32), n_mel)
    np.testing.assert_allclose(sil[:, ::9], g["silence_sub"], atol=1e-5)
    short = log_mel(synth.synth_clip(2, seconds=7.3), n_mel)
    np.testing.assert_allclose(short[:, ::9], g["short_7s_sub"], atol=2e-4)
    assert abs(short.astype(np.float64).sum() - float(g["short_7s_sum"])) < 1e-4 * short.size


def test_encoder_oracle_matches_hf(golden_dir):
    from oracle.encoder import encoder_hidden_states
    g = np.load(os.path.join(golden_dir, "encoder_micro.npz"))
    sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    states = encoder_hidden_states(sd, g["mel"], n_heads=synth.WHISPER_CONFIGS["micro"][3])
    assert len(states) == g["hidden_states"].shape[0]
    for i, s in enumerate(states):
        np.testing.assert_allclose(s, g["hidden_states"][i], atol=2e-4, rtol=2e-4, err_msg=f"hs[{i}]")


def test_decoder_oracle_matches_hf(golden_dir):
    from oracle.decoder import decoder_logits
    g = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    lg = decoder_logits(sd, g["tokens"], g["enc_out"], n_heads=synth.WHISPER_DECODERS["micro"][3])
    np.testing.assert_allclose(np.take_along_axis(lg, g["top_i"], 1), g["top_v"], rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(np.argsort(-lg, axis=1)[:, :5], g["top_i"][:, :5])
    np.testing.assert_allclose(lg[-1], g["logits_last"], atol=2e-4)


def test_cross_attn_oracle_matches_hf(golden_dir):
    """oracle.decoder.cross_attn_probs (the token-level timestamps' input) against transformers 5.15's cross_attentions
    (eager attention, output_attentions=True) of the micro decoder on decoder_micro.npz's encoder output and tokens,
    every (layer, head)."""
    import torch
    from transformers import WhisperConfig, WhisperForConditionalGeneration
    from oracle.decoder import cross_attn_probs
    g = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    V, d, nl, nh, ffn = synth.WHISPER_DECODERS["micro"]
    n_mel, ed, enl, enh, effn = synth.WHISPER_CONFIGS["micro"]
    cfg = WhisperConfig(vocab_size=V, num_mel_bins=n_mel, d_model=d, encoder_layers=enl, encoder_attention_heads=enh,
                        encoder_ffn_dim=effn, decoder_layers=nl, decoder_attention_heads=nh, decoder_ffn_dim=ffn,
                        max_source_positions=1500, max_target_positions=448)
    cfg._attn_implementation = "eager"
    model = WhisperForConditionalGeneration(cfg)
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    model.model.decoder.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()
    with torch.inference_mode():
        out = model(encoder_outputs=(torch.from_numpy(g["enc_out"])[None],),
                    decoder_input_ids=torch.from_numpy(g["tokens"])[None].long(), output_attentions=True)
    heads = [[l, h] for l in range(nl) for h in range(nh)]
    ours = cross_attn_probs(sd, g["tokens"], g["enc_out"], nh, heads)
    ref = np.stack([out.cross_attentions[l][0, h].double().numpy() for l, h in heads])
    np.testing.assert_allclose(ours, ref, rtol=1e-4, atol=1e-7)


def suppression_bias(V, suppress, begin_pos, eos=50257):
    """SuppressTokens (always) + SuppressTokensAtBegin([220, eos]) at the first free position."""
    base = np.zeros(V)
    base[list(suppress)] = -np.inf
    begin = base.copy()
    begin[[220, eos]] = -np.inf
    return lambda pos: begin if pos == begin_pos else base


def test_beam_search_restatement_matches_hf(golden_dir):
    """cbw.generate.beam_search driven by the numpy decoder oracle reproduces HF's beam
    search (num_beams=5) token for token.  HF 5.15 counts generated_len from the
    decoder prompt (decoder_prompt_len = len(prefix)); the build's default is the
    pinned 4.37.2 rule (decoder_prompt_len = 1, pba_whisper forced-ids path)."""
    from cbw.generate import beam_search
    from oracle.decoder import oracle_step_fn
    g = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    prefix = g["beam_prefix"].tolist()
    V = synth.WHISPER_DECODERS["micro"][0]
    bias_at = suppression_bias(V, g["suppress"].tolist(), len(prefix))
    step = oracle_step_fn(sd, g["enc_out"], synth.WHISPER_DECODERS["micro"][3], 10, bias_at)
    out = beam_search(step, prefix, num_beams=5, eos=50257, max_length=len(prefix) + 24,
                      decoder_prompt_len=len(prefix))
    assert out == g["beam_out"].tolist()   # the whole sequence: prefix + all 24 new tokens


@pytest.mark.parametrize("ts", [False, True])
@pytest.mark.parametrize("num_beams", [1, 5])
def test_free_language_position_matches_hf(golden_dir, num_beams, ts):
    """Short-form language=None (4.37.2 forced_decoder_ids (1, None)): the search picks the
    position after <|startoftranscript|> over the whole vocabulary and the task / notimestamps tokens after it stay
    forced -- cbw.generate greedy / beam_search with ``forced`` over the float64 decoder oracle reproduces the HF
    fixture (tests/golden/free_language_micro.npz: ForceTokensLogitsProcessor restated as a processor, the timestamp
    processor also at the free position) token for token."""
    from cbw.generate import beam_search, greedy
    from model.pba_whisper import free_language_positions
    from oracle.decoder import oracle_step_fn
    g = np.load(os.path.join(golden_dir, "free_language_micro.npz"))
    d = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    init = [50258, 50259, 50359] + ([] if ts else [50363])   # language placeholder 50259
    head = g["head"].tolist()
    free = free_language_positions(head[:-1] + init, init)
    assert free["pos"] == len(head) and head[-1] == 50258
    V = synth.WHISPER_DECODERS["micro"][0]
    bias_at = suppression_bias(V, g["suppress"].tolist(), free["begin"])
    rules = (50364, 50363, 50257, 50) if ts else None
    step = oracle_step_fn(sd, d["enc_out"], synth.WHISPER_DECODERS["micro"][3], 2 * num_beams, bias_at, rules,
                          free["begin"], free_pos=free["pos"])
    if num_beams == 1:
        out = greedy(step, head, 50257, len(head) + 24, forced=free["forced"])
    else:
        out = beam_search(step, head, num_beams, 50257, len(head) + 24, decoder_prompt_len=len(head),
                          forced=free["forced"])
    ref = g[f"out_b{num_beams}_ts{int(ts)}"].tolist()
    assert out == ref
    assert all(out[p] == t for p, t in free["forced"].items())


GEN_CASES = ["b5_length_penalty_nrs3", "b5_repetition_penalty", "b5_no_repeat_ngram", "b1_repetition_penalty",
             "b1_no_repeat_ngram", "b4_max_length", "b1_eos_at_5", "b3_eos_at_5"]


@pytest.mark.parametrize("case", GEN_CASES)
def test_generation_controls_restatement_matches_hf(golden_dir, case):
    """A caller's length_penalty / num_return_sequences / repetition_penalty / no_repeat_ngram_size / max_length
    (forwarded to transformers by the reference, pba_whisper.py:320-331) and a hypothesis that
    ends on EOS before max_length (HF writes the EOS back into the output): cbw.generate greedy / beam_search over
    the float64 decoder oracle with the processors restated (oracle_processed_step_fn) reproduce the transformers
    fixture token for token (tests/golden/gen_controls_micro.npz, every returned sequence)."""
    from cbw.generate import beam_search, greedy
    from oracle.decoder import oracle_processed_step_fn
    g = np.load(os.path.join(golden_dir, "gen_controls_micro.npz"))
    d = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    prefix = g["prefix"].tolist()
    V = synth.WHISPER_DECODERS["micro"][0]
    nb = int(case[1])
    ref = g[case]
    eos_case = case.endswith("eos_at_5")
    rp = 1.5 if "repetition" in case else None
    ng = 2 if "ngram" in case else 0
    lp = 0.6 if "length_penalty" in case else 1.0
    nrs = 3 if "nrs3" in case else 1
    new = 12 if eos_case else 24
    max_length = len(prefix) + (10 if "max_length" in case else new)
    if eos_case:   # the fixture's processor: +30 on EOS at one position, no begin suppression
        base = np.zeros(V)
        base[g["suppress"].tolist()] = -np.inf
        boost = base.copy()
        boost[50257] += 30.0
        bias_at = lambda pos: boost if pos == len(prefix) + 5 else base   # noqa: E731
    else:
        bias_at = suppression_bias(V, g["suppress"].tolist(), len(prefix))
    step = oracle_processed_step_fn(sd, d["enc_out"], synth.WHISPER_DECODERS["micro"][3], 2 * nb, bias_at, rp, ng,
                                    greedy=nb == 1)
    if nb == 1:
        out = [greedy(step, prefix, 50257, max_length)]
    else:
        out = beam_search(step, prefix, nb, 50257, max_length, length_penalty=lp, decoder_prompt_len=len(prefix),
                          num_return_sequences=nrs)
        out = out if nrs > 1 else [out]
    assert [list(r) for r in out] == ref.tolist()


def test_beam_sample_restatement_matches_hf(golden_dir):
    """cbw.generate.beam_sample (do_sample with num_beams > 1: processors, temperature / top-k warpers, + beam scores,
    2 num_beams draws without replacement over all beams x vocab, BeamSearchScorer) driven by the float64 decoder
    oracle with a CPU generator seeded as transformers' global RNG reproduces HF's beam-sample output token for token
    (tests/golden/beam_sample_micro.npz, three seeds; EOS suppressed there, see make_golden.make_beam_sample) up to
    the last step.  There the two versions differ by design: at max_length every draw is finished; transformers 5.15
    keeps the first num_beams draws in draw order as the hypotheses, 4.37.2 (restated) sorts the draws by score and
    keeps the best num_beams.  So HF's sequence is the best-scored of the first num_beams draws of our last step, and
    ours the best-scored draw overall -- both on our own trajectory, which therefore followed HF's to the last step.
    The fixture comes from transformers 5.15, whose warpers act on the log-probs before the beam scores are added, so
    the restatement runs in that order here (``warp_order="5.x"``); the product's 4.37.2 order (beam scores first,
    then the warpers) is pinned by test_beam_sample_437_recurrence below."""
    import torch
    from cbw.generate import beam_sample
    from oracle.decoder import oracle_scores_fn
    g = np.load(os.path.join(golden_dir, "beam_sample_micro.npz"))
    d = np.load(os.path.join(golden_dir, "decoder_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    prefix = g["prefix"].tolist()
    V = synth.WHISPER_DECODERS["micro"][0]
    bias_at = suppression_bias(V, g["suppress"].tolist(), len(prefix))
    for seed, hf in zip(g["seeds"].tolist(), g["out"].tolist()):
        fn = oracle_scores_fn(sd, d["enc_out"], synth.WHISPER_DECODERS["micro"][3], bias_at)
        gen = torch.Generator().manual_seed(int(seed))
        nb, tr = int(g["num_beams"]), []
        out = beam_sample(fn, prefix, nb, 50257, len(prefix) + int(g["max_new_tokens"]), float(g["temperature"]),
                          generator=gen, top_k=int(g["top_k"]), decoder_prompt_len=len(prefix), trace=tr,
                          warp_order="5.x")
        assert len(tr) == int(g["max_new_tokens"])
        last = tr[-1]
        s5, r5, t5 = max(last["draws"][:nb], key=lambda c: c[0])    # transformers 5.15: draw order
        s4, r4, t4 = max(last["draws"], key=lambda c: c[0])         # 4.37.2: sorted by score
        assert hf == last["seqs"][r5] + [t5], f"seed {seed}"
        assert out == last["seqs"][r4] + [t4], f"seed {seed}"


def test_beam_sample_437_recurrence():
    """transformers 4.37.2 ``_beam_sample`` (the version the reference pins, requirements.txt:21), restated here line by
    line as an independent loop: processed log-probs + beam scores, THEN the warpers (temperature, top-k) on the sum,
    softmax over num_beams x V, torch.multinomial(2 num_beams), the drawn warped sums sorted -> the next beams and beam
    scores.  cbw.generate.beam_sample (default warp_order "4.37") must draw the same continuations and carry the same
    beam scores at every step (EOS suppressed, so BeamSearchScorer keeps the first num_beams sorted draws), and the
    5.x order must differ (the warpers then act before the beam scores are added)."""
    import torch
    from cbw.generate import beam_sample
    V, nb, T, k, steps, eos = 40, 3, 0.7, 7, 6, 39

    def table(seq):   # a deterministic toy decoder: log-probs of the next token given the row's sequence
        g = torch.Generator().manual_seed(1000003 * len(seq) + sum((i + 1) * t for i, t in enumerate(seq)))
        lp = torch.log_softmax(3.0 * torch.randn(V, generator=g, dtype=torch.float64), -1).float()
        lp[eos] = float("-inf")
        return lp

    class Fn:
        def __init__(self, prefix):
            self.rows = [list(prefix)] * nb

        def __call__(self, tokens, pos, reorder):
            rows = self.rows if reorder is None else [self.rows[r] for r in reorder]
            self.rows = [r + [t] for r, t in zip(rows, tokens)]
            return torch.stack([table(r) for r in self.rows])

    prefix = [5, 9, 2]
    for seed in (0, 1, 2):
        fn = Fn([])
        tr = []
        out = beam_sample(fn, prefix, nb, eos, len(prefix) + steps, T, generator=torch.Generator().manual_seed(seed),
                          top_k=k, decoder_prompt_len=len(prefix), trace=tr)
        gen = torch.Generator().manual_seed(seed)
        seqs, bs = [list(prefix)] * nb, torch.tensor([0.0] + [-1e9] * (nb - 1))
        for j in range(steps):
            assert tr[j]["seqs"] == seqs and np.allclose(tr[j]["beam_scores"], bs.numpy(), rtol=1e-6), (seed, j)
            sc = (torch.stack([table(q) for q in seqs]) + bs[:, None]) / T          # + beam_scores, then warpers
            kth = torch.topk(sc, k, dim=-1).values[:, -1:]
            sc = sc.masked_fill(sc < kth, float("-inf")).view(1, -1)
            nt = torch.multinomial(torch.softmax(sc, -1), 2 * nb, generator=gen)
            ns, order = torch.sort(sc.gather(1, nt), descending=True, dim=1)
            nt = nt.gather(1, order)
            seqs = [seqs[int(t) // V] + [int(t) % V] for t in nt[0, :nb]]
            bs = ns[0, :nb].clone()
        assert out == seqs[int(torch.argmax(bs))], seed
    fn = Fn([])
    tr5 = []
    beam_sample(fn, prefix, nb, eos, len(prefix) + steps, T, generator=torch.Generator().manual_seed(0), top_k=k,
                decoder_prompt_len=len(prefix), trace=tr5, warp_order="5.x")
    fn = Fn([])
    tr4 = []
    beam_sample(fn, prefix, nb, eos, len(prefix) + steps, T, generator=torch.Generator().manual_seed(0), top_k=k,
                decoder_prompt_len=len(prefix), trace=tr4)
    assert not np.allclose(tr4[2]["beam_scores"], tr5[2]["beam_scores"])


def test_language_detection_oracle_matches_hf(golden_dir):
    """detect_language (transformers 5.15, tests/golden/language_micro.npz): the oracle mel -> encoder -> decoder after
    <|startoftranscript|> gives HF's language logits, and their argmax is HF's detected language token."""
    from oracle.decoder import decoder_logits
    from oracle.encoder import encoder_hidden_states
    from oracle.mel import log_mel
    g = np.load(os.path.join(golden_dir, "language_micro.npz"))
    n_mel, _, _, nh, _ = synth.WHISPER_CONFIGS["micro"]
    esd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    dsd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    for c, lid, ref in zip(g["clips"].tolist(), g["lang_ids"].tolist(), g["lang_logits"]):
        enc = encoder_hidden_states(esd, log_mel(synth.synth_clip(c), n_mel), nh)[-1]
        lg = decoder_logits(dsd, [50258], enc, synth.WHISPER_DECODERS["micro"][3], last_only=True)[0]
        lang = lg[50259:50259 + 99]
        np.testing.assert_allclose(lang, ref, rtol=1e-3, atol=1e-3 * np.abs(ref).max())
        assert 50259 + int(np.argmax(lang)) == lid


# ---- the torch-fp32 restatement bench.py's cpu_baseline times (oracle/torch_ref.py) ----

@pytest.mark.parametrize("name", ["LEF", "LE", "LEF_r18"])
def test_torch_ref_kws_matches_reference_golden(name, golden_dir):
    import oracle.torch_ref as tref
    hp, bk = KWS_CASES[name]
    g = np.load(os.path.join(golden_dir, f"kws_{name}.npz"))
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
    logits = tref.kws_forward(sd, hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], group=3).numpy()
    np.testing.assert_allclose(logits, g["logits"], rtol=1e-3, atol=1e-3 * np.abs(g["logits"]).max())


def test_torch_ref_mel_and_encoder_match_hf(golden_dir):
    import torch
    import oracle.torch_ref as tref
    g = np.load(os.path.join(golden_dir, "mel_80.npz"))
    np.testing.assert_allclose(tref.log_mel(synth.synth_clip(0), 80).numpy(), g["noise_sines"], atol=2e-4)
    e = np.load(os.path.join(golden_dir, "encoder_micro.npz"))
    sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    states = tref.encoder_hidden_states(sd, torch.from_numpy(e["mel"]), synth.WHISPER_CONFIGS["micro"][3])
    for i, s in enumerate(states):
        np.testing.assert_allclose(s.numpy(), e["hidden_states"][i], atol=1e-3, rtol=1e-3, err_msg=f"hs[{i}]")


def test_long_form_mel_oracle_matches_hf():
    """oracle.mel.log_mel_long == WhisperFeatureExtractor(padding='longest', truncation=False) on 77 s."""
    from oracle.mel import log_mel_long
    fe = pytest.importorskip("transformers").WhisperFeatureExtractor
    x = np.concatenate([synth.synth_clip(i) for i in range(3)])[:1234567]
    for n_mel in (80, 128):
        ref = fe(feature_size=n_mel)(x, sampling_rate=16000, padding="longest", truncation=False,
                                     return_tensors="np")["input_features"][0]
        np.testing.assert_allclose(log_mel_long(x, n_mel), ref, atol=1e-4)


def test_padded_prompt_rows_oracle_beam_search_matches_hf_batch(golden_dir):
    """The batched long-form loop's left-padded decoder inputs (pba_whisper.py:478-548; transformers 4.37.2 passes
    decoder_attention_mask=None to the decoder, so the pads are attended as tokens at their positions):
    tests/golden/padded_beams_micro.npz holds HF's beam search (5 beams) over three such rows as one batch without a
    decoder mask; cbw.generate.beam_search driven by the float64 decoder oracle on each padded row alone reproduces
    each batch row token for token (batch elements are independent; the pads are ordinary tokens)."""
    from cbw.generate import beam_search
    from oracle.decoder import oracle_step_fn
    g = np.load(os.path.join(golden_dir, "padded_beams_micro.npz"))
    sd = synth.synth_whisper_decoder_state_dict("micro", seed=0)
    V = synth.WHISPER_DECODERS["micro"][0]
    rows = g["rows"].tolist()
    L = len(rows[0])
    for i, row in enumerate(rows):
        assert 50257 in row[1:] or i == 1   # rows 0 and 2 are padded (row 1 is the longest prompt)
        step = oracle_step_fn(sd, g["enc_out"][i], synth.WHISPER_DECODERS["micro"][3], 10,
                              suppression_bias(V, g["suppress"].tolist(), L))
        out = beam_search(step, row, num_beams=5, eos=50257, max_length=L + 24, decoder_prompt_len=L)
        hf = g["out"][i].tolist()
        assert out == hf[:len(out)] and all(t == 50257 for t in hf[len(out):]), f"row {i}"
