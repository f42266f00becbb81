"""CPU: the CLI mirrors keep the reference scripts' flags, defaults, types and choices
(tests/golden/cli_flags.json, recorded from the reference by make_cli_golden.py)."""
import importlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS_DIR = os.path.join(ROOT, "vae-diffusion-toy-crystals_amd", "scripts")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from make_cli_golden import describe  # noqa: E402  (shared describer; no reference import at module level)


# flags a mirror adds on top of the reference's (additive only: every reference flag is kept as is)
ADDITIVE = {"build_dataset": {"device", "render_batch"}, "train_sde_score_model": {"global_draws"},
            "train_vae": {"global_draws", "replay_draws"}, "train_diffusion_prior": {"global_draws", "zero"}}


@pytest.mark.parametrize("name", ["train_sde_score_model", "sample_sde_score_model", "train_vae",
                                  "train_diffusion_prior", "build_dataset"])
def test_cli_matches_reference(name):
    with open(os.path.join(ROOT, "tests", "golden", "cli_flags.json")) as f:
        ref = json.load(f)[name]
    if SCRIPTS_DIR not in sys.path:
        sys.path.insert(0, SCRIPTS_DIR)
    mod = importlib.import_module(name)
    mine = json.loads(json.dumps(describe(mod.build_parser()), default=str))
    mine = [d for d in mine if d["dest"] not in ADDITIVE.get(name, set())]
    assert mine == ref
