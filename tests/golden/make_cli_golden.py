#!/usr/bin/env python3
"""Record the reference CLIs' flags and defaults (tests/golden/cli_flags.json).

Run ONLY in the build container:
    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src:/root/reference python tests/golden/make_cli_golden.py
Each reference script's main() builds its argparse parser and calls parse_args(); parse_args is
intercepted to capture the parser and stop before anything else runs.
"""
import argparse
import importlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPTS = ["train_sde_score_model", "sample_sde_score_model", "train_vae", "train_diffusion_prior", "build_dataset"]


class _Captured(Exception):
    pass


def describe(parser: argparse.ArgumentParser):
    out = []
    for a in parser._actions:
        if isinstance(a, argparse._HelpAction):
            continue
        out.append({"options": sorted(a.option_strings), "dest": a.dest, "default": a.default,
                    "type": getattr(a.type, "__name__", None), "choices": list(a.choices) if a.choices else None,
                    "required": bool(a.required), "action": type(a).__name__})
    return sorted(out, key=lambda d: (d["dest"], d["options"]))


def capture(modname: str):
    mod = importlib.import_module("scripts." + modname)
    got = {}
    orig = argparse.ArgumentParser.parse_args

    def fake(self, *a, **k):
        got["p"] = self
        raise _Captured()
    argparse.ArgumentParser.parse_args = fake
    try:
        mod.main()
    except _Captured:
        pass
    finally:
        argparse.ArgumentParser.parse_args = orig
    return describe(got["p"])


def main():
    res = {name: capture(name) for name in SCRIPTS}
    with open(os.path.join(HERE, "cli_flags.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True, default=str)
    print("wrote cli_flags.json", {k: len(v) for k, v in res.items()})


if __name__ == "__main__":
    sys.exit(main())
