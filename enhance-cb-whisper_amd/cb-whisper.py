"""Entry point with the reference's CLI shape (src/cb-whisper.py:1-13):

    python cb-whisper.py test --config configs/cb-whisper-acl.yaml [--model.init_args.root=/data/acl ...]

The reference hands the YAML to LightningCLI (``subclass_mode_model=True``), which builds
``model.class_path`` (model.cb_whisper.CBWhisper) from ``model.init_args`` and runs ``trainer.test`` over
``data.class_path`` (data.data_module.KWSDataMod).  This runner reads the same file unchanged
(cbw.cli: ``class_path``/``init_args``, dotted overrides for the published ``[PLACEHOLDER]`` values) and
builds the same CBWhisper -- checkpoints are local HF-format directories (cbw.checkpoint).  The ACL/Aishell
audio + transcript loaders (data/dataset.py) are dataset I/O, out of scope: ``--synthetic N`` runs N seeded
30 s clips through ``test_step`` / ``on_test_epoch_end`` (mel -> spotting -> prompt -> beam search on the
GPU) so the YAML -> model -> GPU path runs end to end; without it the runner builds the model and reports
it.  ``fit``/``validate`` are training and out of scope.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

os.environ.setdefault("OMP_NUM_THREADS", "2")   # cb-whisper.py:2

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def main(argv=None):
    from cbw import cli
    argv = list(sys.argv[1:] if argv is None else argv)
    own, overrides = cli.split_argv(argv, ("--config", "--synthetic", "--seed", "--max-new-tokens"))
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("subcommand", choices=["test", "fit", "validate"])
    ap.add_argument("--config", required=True)
    ap.add_argument("--synthetic", type=int, default=0, help="run N seeded synthetic 30 s clips through test_step")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-new-tokens", type=int, default=None)
    sub = [a for a in overrides if not a.startswith("--")][:1]
    args = ap.parse_args(sub + own)
    overrides = [a for a in overrides if a not in sub]
    if args.subcommand != "test":
        raise SystemExit(f"'{args.subcommand}' is training and out of scope for the MI355X inference path")
    cfg = cli.load_config(args.config, overrides)
    missing = cli.placeholders(cfg["model"])
    if missing:
        raise SystemExit("set the config placeholders first, e.g. " +
                         " ".join(f"--model.init_args.{k}=..." for k in missing))
    model = cli.build(cfg["model"])
    if not args.synthetic:
        print(json.dumps({"model": type(model).__name__, "keywords": len(model.keywords),
                          "hparams": {k: str(v) for k, v in vars(model.hparams).items()},
                          "note": "model built from the YAML; dataset I/O (data.data_module) is out of scope: "
                                  "use --synthetic N to run clips end to end"}))
        return 0
    import torch
    from cbw import synth
    from cbw.whisper import log_mel
    if args.max_new_tokens is not None:   # bound the beam search of the synthetic run
        gen = model.whisper.generate
        model.whisper.generate = lambda *a, **k: gen(*a, max_new_tokens=args.max_new_tokens, **k)
    model.on_test_epoch_start()
    n_mel = model.whisper.encoder_config[0]
    out = []
    for i in range(args.synthetic):
        clip = torch.from_numpy(synth.synth_clip(args.seed + i)).to(model.whisper.device)
        mel, _ = log_mel(clip, n_mel)
        batch = {"utterance": {"features": mel[None], "attention_mask": None}, "transcript": "",
                 "speaker": "synthetic", "hotword_labels": [torch.zeros(len(model.keywords), dtype=torch.long)]}
        r = model.test_step(batch, i)
        out.append({"clip": i, "spotted": model.last_spotted[0] if model.last_spotted else [], "pred": r["preds"]})
    print(json.dumps({"results": out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
