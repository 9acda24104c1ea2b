"""The slice of LightningCLI / jsonargparse the reference entry points use (src/cb-whisper.py:1-13,
src/run_efficient_kws.py:9-55): a YAML config with ``model`` / ``data`` sections in ``class_path`` +
``init_args`` form, dotted command-line overrides (``--model.init_args.root=/data/acl``), and the published
configs' ``[PLACEHOLDER]`` values (README.md:143), which YAML reads as one-element lists of an upper-case
string.  Neither Lightning nor jsonargparse is installed, so this is what builds the models from the
unchanged YAML files.
"""
from __future__ import annotations

import importlib
from typing import Iterable, List, Tuple

import yaml


def is_placeholder(v) -> bool:
    """``[ACL_ROOT]`` / ``[MODALITY(tts/natural)]`` -> ['ACL_ROOT'] after YAML parsing."""
    return isinstance(v, list) and len(v) == 1 and isinstance(v[0], str) and v[0][:1].isupper() and \
        v[0].split("(")[0].replace("_", "").isupper()


def apply_overrides(cfg: dict, args: Iterable[str]) -> dict:
    """``--a.b.c=value`` / ``--a.b.c value`` (value parsed as YAML, as jsonargparse does)."""
    args = list(args)
    i = 0
    while i < len(args):
        a = args[i]
        if not a.startswith("--") or "." not in a.split("=")[0]:
            raise SystemExit(f"unrecognised argument {a!r} (expected --section.key=value)")
        if "=" in a:
            key, val = a[2:].split("=", 1)
            i += 1
        else:
            if i + 1 >= len(args):
                raise SystemExit(f"missing value for {a}")
            key, val = a[2:], args[i + 1]
            i += 2
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = yaml.safe_load(val)
    return cfg


def load_config(path: str, overrides: Iterable[str] = ()) -> dict:
    with open(path) as f:
        cfg = yaml.safe_load(f)
    return apply_overrides(cfg, overrides)


def placeholders(section: dict) -> List[str]:
    return [k for k, v in (section.get("init_args") or {}).items() if is_placeholder(v)]


def build(section: dict, drop_placeholders: bool = False):
    """Instantiate ``class_path`` with ``init_args`` (placeholders dropped -> the class default, or kept and
    reported by the caller)."""
    mod, cls = section["class_path"].rsplit(".", 1)
    init = dict(section.get("init_args") or {})
    if drop_placeholders:
        init = {k: v for k, v in init.items() if not is_placeholder(v)}
    return getattr(importlib.import_module(mod), cls)(**init)


def split_argv(argv: List[str], known: Tuple[str, ...]) -> Tuple[List[str], List[str]]:
    """Separate this runner's own flags (``known``, each taking one value unless it is a switch ending in
    '!') from the dotted config overrides."""
    own, rest = [], []
    i = 0
    flags = {k.rstrip("!"): k.endswith("!") for k in known}
    while i < len(argv):
        a = argv[i]
        name = a.split("=")[0]
        if name in flags:
            own.append(a)
            if not flags[name] and "=" not in a and i + 1 < len(argv):
                own.append(argv[i + 1])
                i += 1
        else:
            rest.append(a)
        i += 1
    return own, rest
