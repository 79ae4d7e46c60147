"""Lane occupancy of the Huffman lane pass (k_inflate_tokens) from tools/lane_sim.c's per-block
iteration counts: blocks go to lanes in order, 64 per wave, and a wave runs each DEFLATE-block
phase until its slowest lane ends it (the per-phase headers are decoded by all lanes together), so
its time is the sum over phases of the phase's longest lane.  Occupancy = lane-iterations of work
/ (64 x the wave's iterations).

    gcc -O2 -o /tmp/lane_sim tools/lane_sim.c && /tmp/lane_sim FILE.bam 20000 > blocks.txt
    python tools/lane_sim.py blocks.txt
"""
import sys

import numpy as np


def main():
    rows = [list(map(int, l.split())) for l in open(sys.argv[1])]
    rows = [r for r in rows if r[2] > 0]
    P = max(r[2] for r in rows)
    it = np.zeros((len(rows), P))
    for i, r in enumerate(rows):
        it[i, :r[2]] = r[3:3 + r[2]]
    n = len(rows) // 64 * 64
    it = it[:n]
    W = it.reshape(-1, 64, P)
    wave = W.max(1).sum(1)
    tot = it.sum(1)
    print("blocks %d, %d phases max; iterations per block mean %.0f std %.0f (phase 0 %.0f, phase 1 %.0f)"
          % (n, P, tot.mean(), tot.std(), it[:, 0].mean(), it[:, 1].mean() if P > 1 else 0))
    print("lane occupancy, blocks in file order: %.4f" % (W.sum() / (64 * wave.sum())))
    print("lane occupancy if the phases were flattened: %.4f" % (tot.sum() / (64 * tot.reshape(-1, 64).max(1).sum())))


if __name__ == "__main__":
    main()
