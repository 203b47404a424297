"""Writes tests/golden/hybrid_test_fork.json from the fork's captured output
/root/reference/hybrid_test.txt (run once, in the build container; the GPU
box has no /root/reference).

The file is the output of the fork's HybridGridTest.wang
(mapping/3d/hybrid_grid_test.cc:119-150) run at resolutions 1.0, 2.0 and 3.0:
eight points (:121-125, stated here as the test states them) are set to
probability 1 (kept as kMaxProbability 0.9) at HybridGrid::GetCellIndex;
the grid's iterator then yields (cell index, probability) and an
InterpolatedProbabilityGrid is evaluated at point + (float(0.2 * i), 0, 0),
point = (-7, 3, 1), i = 1..19, next to the probability of the point's cell.
Values were printed with std::cout's 6 significant digits. The fixture keeps
the inputs and the expected outputs only.

    python tests/golden/make_hybrid_fixture.py [/root/reference/hybrid_test.txt]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
POINTS = [(-3.0, 2.0, 0.0), (-4.0, 2.0, 0.0), (-5.0, 2.0, 0.0), (-6.0, 2.0, 0.0),
          (-6.0, 3.0, 1.0), (-6.0, 4.0, 2.0), (-7.0, 3.0, 1.0), (-1.0, 3.0, 1.0)]
SAMPLE_ORIGIN = (-7.0, 3.0, 1.0)


def parse(text):
    sections = []
    cur = None
    for line in text.splitlines():
        line = line.strip()
        m = re.match(r"resolution:?\s*([0-9.]+)f", line)
        if m:
            cur = {"resolution": float(m.group(1)), "cells": [], "samples": []}
            sections.append(cur)
            continue
        m = re.match(r"cell index:\s*(-?\d+),\s*(-?\d+),(-?\d+) prob: ([0-9.]+)", line)
        if m:
            cur["cells"].append({"index": [int(m.group(i)) for i in (1, 2, 3)],
                                 "probability": float(m.group(4))})
            continue
        m = re.match(r"cell (-?[0-9.]+),(-?[0-9.]+),(-?[0-9.]+) prob: ([0-9.]+)", line)
        if m:
            cur["samples"].append({"printed_point": [float(m.group(i)) for i in (1, 2, 3)],
                                   "cell_probability": float(m.group(4))})
            continue
        m = re.match(r"interpolated: ([0-9.]+)", line)
        if m:
            cur["samples"][-1]["interpolated"] = float(m.group(1))
    return sections


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/hybrid_test.txt"
    sections = parse(open(src).read())
    for s in sections:
        assert len(s["samples"]) == 19 and all("interpolated" in x for x in s["samples"]), s
        for i, x in enumerate(s["samples"], start=1):
            x["i"] = i  # point = SAMPLE_ORIGIN + (float(0.2 * i), 0, 0), float adds
    out = {"source": "fork output /root/reference/hybrid_test.txt of HybridGridTest.wang "
                     "(mapping/3d/hybrid_grid_test.cc:119-150)",
           "points": POINTS, "probability_set": 1.0, "sample_origin": SAMPLE_ORIGIN,
           "sample_step": 0.2, "printed_significant_digits": 6, "sections": sections}
    path = os.path.join(HERE, "hybrid_test_fork.json")
    json.dump(out, open(path, "w"), indent=1)
    print(f"wrote {path}: " + ", ".join(f"res {s['resolution']}: {len(s['cells'])} cells"
                                        for s in sections))


if __name__ == "__main__":
    main()
