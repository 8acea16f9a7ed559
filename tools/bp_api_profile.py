#!/usr/bin/env python3
"""cProfile of BeliefPropagation.calibrate() on pathfinder through the compiled schedule (host
overhead around the 0.5 ms graph replay).  python tools/bp_api_profile.py"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from pgmpy_amd.inference import BeliefPropagation
    from pgmpy_amd.utils import get_example_model

    os.environ["PGM_BP_COMPILED"] = "1"
    bp = BeliefPropagation(get_example_model("pathfinder"))
    bp.calibrate()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        bp.calibrate()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
