#!/usr/bin/env python3
"""Notes of the compiled single-query programs of the C1 patterns (alarm): what each launch is."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import collections

    import torch

    from pgmpy_amd.inference import VariableElimination
    from pgmpy_amd.utils import get_example_model
    from pgmpy_amd.utils.sampling import forward_sample_codes

    m = get_example_model("alarm")
    nodes_sorted = sorted(m.nodes())
    rng = random.Random(1)
    codes, nodes = forward_sample_codes(m, 50, seed=1)
    pos = {v: i for i, v in enumerate(nodes)}
    ve = VariableElimination(m)
    for r in range(50):
        pick = rng.sample(nodes_sorted, 8)
        ve.query(pick[:3], {v: m.states[v][codes[pos[v], r]] for v in pick[3:]}, show_progress=False)
    torch.cuda.synchronize()
    shapes = collections.Counter()
    for i, rn in enumerate(ve._compiled.values()):
        for prog, *_ in rn.plan.__dict__.get("_progs", {}).values():
            shapes[tuple(n.split(" [")[0][:60] for n in prog.notes)] += 1
            if i < 3:
                for us, note in prog.time_steps(reps=20):
                    print(f"  {us:6.2f} us  {note[:120]}")
                print("  --", prog.direct_note)
    for k, v in shapes.most_common(8):
        print(v, k)


if __name__ == "__main__":
    main()
