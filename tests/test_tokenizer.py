"""The local Whisper tokenizer (cbw/tokenizer.py) against transformers' WhisperTokenizer on the same files.

The reference calls ``WhisperProcessor.get_prompt_ids`` (src/model/cb_whisper.py:140-147) and
``tokenizer.batch_decode(..., skip_special_tokens=True)`` (:180-186).  No Whisper tokenizer files exist
offline, so both sides read a seeded byte-level BPE vocabulary in the Whisper file layout with the real
special-token ids (cbw.synth.write_synth_tokenizer).  CPU only.
"""
import numpy as np
import pytest

from cbw import synth
from cbw.tokenizer import WhisperTokenizerLite

TEXTS = [
    "The topic of today's speech is, ah, alpha, bravo. Okay, then I'll continue.",
    "keyword spotting  whisper\n x",
    "ünïcode 123 delta-echo",
    "  leading and trailing spaces   ",
    "machine translation, attention, transformer, neural model",
    "",
]


@pytest.fixture(scope="module")
def toks(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("tok"))
    synth.write_synth_tokenizer(d)
    hf = pytest.importorskip("transformers").WhisperTokenizer.from_pretrained(d)
    return WhisperTokenizerLite.from_dir(d), hf


@pytest.mark.parametrize("text", TEXTS)
def test_prompt_ids_match_hf(toks, text):
    lite, hf = toks
    assert lite.get_prompt_ids(text) == [int(x) for x in hf.get_prompt_ids(text)]


def test_prompt_with_special_token_raises_like_hf(toks):
    lite, hf = toks
    for t in ("hello <|en|> x", "a <|0.00|>"):
        with pytest.raises(ValueError):
            hf.get_prompt_ids(t)
        with pytest.raises(ValueError):
            lite.get_prompt_ids(t)


def test_decode_matches_hf(toks):
    lite, hf = toks
    sot, en, tr, nots = (lite.convert_tokens_to_ids(t) for t in
                         ("<|startoftranscript|>", "<|en|>", "<|transcribe|>", "<|notimestamps|>"))
    body = lite.encode(" alpha bravo, the speech is okay.")
    seqs = [[sot, en, tr, nots] + body + [lite.eot],
            lite.get_prompt_ids("delta echo") + [sot, en, tr, nots] + body,
            [sot, en, tr] + [lite.convert_tokens_to_ids("<|0.00|>")] + body + [lite.convert_tokens_to_ids("<|1.20|>")]]
    for s in seqs:
        assert lite.decode(s, skip_special_tokens=True) == hf.decode(s, skip_special_tokens=True)
    assert lite.decode(seqs[0]) == hf.decode(seqs[0])


def test_encode_roundtrip_random_bytes(toks):
    lite, hf = toks
    rng = np.random.default_rng(0)
    for _ in range(20):
        s = "".join(chr(c) for c in rng.integers(32, 0x2ff, 30))
        ids = lite.encode(s)
        assert ids == hf.encode(s, add_special_tokens=False)
        assert lite.decode(ids) == s


def test_eot_in_vocab_is_special_like_hf(toks):
    """vocab.json lists <|endoftext|> (as real Whisper files do) and added_tokens.json too: it stays special --
    greedy outputs end in EOT and decode(skip_special_tokens=True) drops it -- and get_prompt_ids rejects ids from
    all_special_ids[0] (= <|endoftext|>) on, as transformers does."""
    lite, hf = toks
    assert lite.eot == 50257 and lite.first_special == hf.all_special_ids[0] == 50257
    sot, en, tr, nots = (lite.convert_tokens_to_ids(t) for t in
                         ("<|startoftranscript|>", "<|en|>", "<|transcribe|>", "<|notimestamps|>"))
    body = lite.encode(" alpha bravo")
    for s in ([sot, en, tr, nots] + body + [lite.eot], body + [lite.eot, lite.eot]):
        assert lite.decode(s, skip_special_tokens=True) == hf.decode(s, skip_special_tokens=True)
        assert lite.decode(s) == hf.decode(s)
    # timestamps are not special: kept with decode_with_timestamps (as their own text; transformers 5.15 prints
    # them from all_special_ids[-1] + 1, an id its unordered special set no longer pins -- not compared)
    ts = [lite.convert_tokens_to_ids("<|0.00|>")] + body + [lite.convert_tokens_to_ids("<|1.20|>"), lite.eot]
    assert lite.decode(ts, skip_special_tokens=True, decode_with_timestamps=True) == "<|0.00|> alpha bravo<|1.20|>"
    with pytest.raises(ValueError):
        hf.get_prompt_ids("a <|endoftext|> b")
    with pytest.raises(ValueError):
        lite.get_prompt_ids("a <|endoftext|> b")
