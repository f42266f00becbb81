#!/usr/bin/env python3
"""Run one U-Net conv layer shape repeatedly (for rocprofv3 --pmc passes). LAYER=name REPS=n."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PRO", "0")
import convbench as cb  # noqa: E402  (prints the per-layer timings of the selected layer only)
