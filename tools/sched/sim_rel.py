"""Replays record.py --rel records under the held stream (sim.py holdb+face
--par) with the change marks of the relevance rule: none (cur), faces only,
the block's own mark only, both.  usage: sim_rel.py REC.npz KB"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sim  # noqa: E402
R = np.load(sys.argv[1]); kb = int(sys.argv[2])
g = sim.Geo(int(R["nx"]), int(R["ny"]), int(R["nz"]))
sim.PAR = True
nst = len(R["stations"])
for mode in ("cur", "face_only", "own_only", "both"):
    pos = 0
    for k in range(nst):
        chg, face = R[f"chg{k}"], R[f"face{k}"]
        orl, frl = R[f"own_rel{k}"], R[f"face_rel{k}"]
        rel = {"cur": None, "face_only": (chg, frl), "own_only": (orl, face), "both": (orl, frl)}[mode]
        t = sim.run(chg, face, R[f"bc{k}"], g, "holdb+face", kb=kb, infl=1 + -(-16 // kb), vis=-(-12 // kb), rel=rel)
        pos += t["pos"]
    print(mode, pos / nst, flush=True)
