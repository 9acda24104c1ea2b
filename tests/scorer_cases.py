"""Inputs of the entity-recall / tokenizer fixtures (tests/golden/scorer.json).  Data only."""

TOKENIZER_TEXTS = [
    "",
    "Hello world",
    "Dr. Smith went to Washington. He arrived at 5 p.m. today.",
    "Mr. Li said: \"the GPU (MI355X) is fast!\" -- really?\nYes.\n\nNew paragraph here.",
    "价格是 5 元。我们明天见。",
    "ኢትዮጵያ። ሰላም",
    "a | b || c|d",
    "cost $5 + tax = 7€ ... ok. fin",
    "tabs\tand  spaces nbsp end.",
    "trailing symbols $$$",
    "Ends with a stop. ",
    "x. y. longer. word. here",
    "   leading spaces",
    "emoji 🙂 inside 🙂🙂 text",
    "\r\nwindows\r\nlines\r\n",
]

# (pred, ref, mentions) triples; mentions = dicts with total_offset/end_offset (character span in ref)
def _m(ref, word, tag="UNK", nth=0):
    i = -1
    for _ in range(nth + 1):
        i = ref.index(word, i + 1)
    return {"mention": word, "total_offset": i, "end_offset": i + len(word), "ner_tag": tag}


_R1 = "we use the Transformer model with BERT embeddings"
_R2 = "Smith and Wesson met John Smith in Paris"
_R3 = "the ACL conference in Dublin"
_R4 = "价格是五元我们明天见北京"
_R5 = "deep | learning on GPUs, the | pipe"
_R6 = "multi word entity recognition systems are here"

RECALL_CASES = [
    # exact transcript
    (_R1, _R1, [_m(_R1, "Transformer", "MISC"), _m(_R1, "BERT", "MISC")]),
    # one entity misspelt, one correct
    ("we use the transformer model with BERT embedding", _R1, [_m(_R1, "Transformer", "MISC"), _m(_R1, "BERT", "ORG")]),
    # empty prediction
    ("   ", _R2, [_m(_R2, "Smith", "PER"), _m(_R2, "Paris", "LOC")]),
    # repeated mention text, overlapping mentions
    ("Smith and Weston met Jon Smith in Paris", _R2,
     [_m(_R2, "Smith", "PER"), _m(_R2, "Smith", "PER", 1), _m(_R2, "Smith and Wesson", "ORG"), _m(_R2, "Paris", "LOC")]),
    # insertions / deletions around the entity
    ("the the ACL big conference in in Dublin city", _R3, [_m(_R3, "ACL", "ORG"), _m(_R3, "Dublin", "LOC")]),
    ("ACL conference", _R3, [_m(_R3, "ACL", "ORG"), _m(_R3, "Dublin", "LOC")]),
    # chinese (char split matters)
    ("价格是五元我们明天见背景", _R4, [_m(_R4, "五元"), _m(_R4, "北京")]),
    # literal pipes in both texts
    ("deep | learning on GPU, the || pipe", _R5, [_m(_R5, "learning"), _m(_R5, "GPUs"), _m(_R5, "pipe")]),
    # multi-token entity with a gap inside the aligned span
    ("multi word entity entity recognition system are here", _R6,
     [_m(_R6, "multi word entity recognition", "MISC"), _m(_R6, "systems", "MISC")]),
    # no mentions
    ("anything", "something else", []),
]

NER_TAG_SETS = ["ALL", ["MISC"], ["PER", "LOC"], ["UNK", "ORG"]]
