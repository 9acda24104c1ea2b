"""Entry point with the reference's CLI shape (src/run_efficient_kws.py:9-55):

    python run_efficient_kws.py test --config efficient_kws/configs/eval-LEF-comp-acl.yaml [--ckpt_path X]

The reference builds everything through LightningCLI + jsonargparse; neither is
installed here, so this runner reads the same YAML files (yaml.safe_load), builds
``model.class_path`` (efficient_kws.model.KWSModel) from ``model.init_args`` exactly
as the CLI would, restores ``ckpt_path`` (Lightning .ckpt, weights_only load) and runs
``test_step`` over the data.  Dataset I/O (``efficient_kws.data_module.KWSDataMod``,
corpora, hs .bin files) is out of scope; without ``--synthetic`` the runner stops
after building the model, with ``--synthetic`` it scores seeded synthetic batches
(cbw.synth) so the YAML -> model -> GPU path is exercised end to end.  ``fit`` is
training and out of scope.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

os.environ.setdefault("OMP_NUM_THREADS", "2")   # run_efficient_kws.py:3

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def build_model(cfg: dict):
    mcfg = cfg["model"]
    mod, cls = mcfg["class_path"].rsplit(".", 1)
    init = dict(mcfg.get("init_args", {}))
    for k, v in list(init.items()):
        if isinstance(v, list) and len(v) == 1 and isinstance(v[0], str) and v[0].isupper():
            init.pop(k)          # "[PLACEHOLDER]" values of the published YAMLs (README.md:143)
    return getattr(importlib.import_module(mod), cls)(**init)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("subcommand", choices=["test", "fit", "validate"])
    ap.add_argument("--config", required=True)
    ap.add_argument("--ckpt_path", default=None)
    ap.add_argument("--synthetic", type=int, default=0, help="score N seeded synthetic utterances")
    ap.add_argument("--keywords", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    if args.subcommand != "test":
        raise SystemExit(f"'{args.subcommand}' is training and out of scope for the MI355X inference path")
    import yaml
    with open(args.config) as f:
        cfg = yaml.safe_load(f)
    model = build_model(cfg)
    ckpt = args.ckpt_path or cfg.get("ckpt_path")
    if isinstance(ckpt, str) and os.path.exists(ckpt):
        model = type(model).load_from_checkpoint(ckpt)
    elif args.synthetic:
        from cbw import synth
        hp = vars(model.hparams)
        model.load_state_dict(synth.synth_kws_state_dict(seed=args.seed, **{k: hp[k] for k in (
            "n_layers", "embedding_dim", "learn_features", "proj_mlp", "frames_conv", "proj_mlp_units",
            "resnet_version")}))
    else:
        print(json.dumps({"model": type(model).__name__, "hparams": {k: str(v) for k, v in vars(model.hparams).items()},
                          "note": "no checkpoint/data: model built from YAML only"}))
        return 0
    if not args.synthetic:
        raise SystemExit("real datasets (KWSDataMod) are out of scope; use --synthetic N")
    import torch
    from cbw import synth
    hp = vars(model.hparams)
    tk, tu = tuple(hp.get("features_size", (150, 1500)))
    results = []
    for i in range(args.synthetic):
        b = synth.synth_kws_batch(seed=args.seed + i, K=args.keywords, n_layers=hp["n_layers"],
                                  D=hp["embedding_dim"], Tk=tk, Tu=tu, plant=(0,))
        batch = {"kwd": [torch.from_numpy(b["kwd"])], "kwd_mask": [torch.from_numpy(b["kwd_mask"])],
                 "utt": torch.from_numpy(b["utt"][0]), "utt_mask": torch.from_numpy(b["utt_mask"][0]),
                 "hotword_mask": [torch.from_numpy(b["ghost_mask"])],
                 "hotword_labels": [torch.zeros(args.keywords, dtype=torch.long)], "speaker": "synthetic"}
        out = model.test_step(batch, i)
        p = out["preds"].cpu()
        results.append({"utterance": i, "spotted": (p >= float(hp["threshold"])).nonzero().flatten().tolist()})
    print(json.dumps({"threshold": hp["threshold"], "results": results}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
