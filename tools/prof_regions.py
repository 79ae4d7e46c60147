"""Where the cycles go, from the HBAM_PROF build (libhbam_prof.so, s_memtime stamps).

inflate: one hbam_decode_split over a synthetic BAM; per BGZF block the Huffman pass adds its
  cycles per region (slots 16..23 of 32 per block) and counts (24..27):
  regions 0 epoch/stall, 1 lit/len lookup, 2 literal, 3 length extra + refill, 4 distance,
  5 match emit, 6 header/tables, 7 slow path; counts 0 symbols, 1 stalls, 2 slow symbols.
guess: one hbam_guess_batch of --guesses random offsets; per guess 8 slots:
  0 whole guess, 1 BGZF candidate search, 2 BAM candidate search, 3 record chain decode,
  4 BGZF candidates tried, 5 BAM candidates tried, 6 records decoded, 7 listed magics."""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
os.environ["HBAM_LIB"] = os.path.join(ROOT, "hadoop-bam_amd", os.environ.get("PROF_LIB", "libhbam_prof.so"))
os.environ["HBAM_INFLATE_SLICES"] = "1"  # per-block prof slots are indexed per launch
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402


def pct(v):
    return "mean %9.0f p50 %9.0f p90 %9.0f p99 %9.0f max %9.0f" % (
        v.mean(), np.percentile(v, 50), np.percentile(v, 90), np.percentile(v, 99), v.max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["inflate", "guess"])
    ap.add_argument("--size", type=float, default=2e9)
    ap.add_argument("--guesses", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=3)
    a = ap.parse_args()
    g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    data = np.asarray(g)
    n = len(data)
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    d[:n].copy_(torch.from_numpy(data))
    d[n:].zero_()
    torch.cuda.synchronize()
    ctx = _lib.Context(0)
    L = _lib.load()
    h = ctx.parse_header(d[:n])
    if a.mode == "inflate":
        L.hbam_prof_attach.argtypes = [C.c_void_p]
        pbuf = torch.zeros((n // 8000 + 4096) * 32, dtype=torch.int64, device="cuda")
        assert L.hbam_prof_attach(C.c_void_p(pbuf.data_ptr())) == 0
        for _ in range(2):
            pbuf.zero_()
            rc, cols = ctx.decode_split_device(d[:n], h["first_voffset"], (n << 16) | 0xffff, h["n_ref"])
            assert rc == 0 and cols.status == 0, (rc, cols.status if rc == 0 else None, ctx.last_error())
        t = ctx.timing()
        print({k: round(v, 3) if isinstance(v, float) else v for k, v in t.items()}, flush=True)
        nb = t["n_blocks"]
        P = pbuf.view(-1, 32)[:nb].cpu().numpy().astype(np.float64)
        R = P[:, 16:24]
        tot = R.sum()
        names = ["epoch", "symbol loop", "loop latch", "hdr+CL table", "code lengths", "LL+D tables",
                 "drain", "slow path"]
        print("Huffman pass, %d blocks, %.3g cycles summed over lanes" % (nb, tot))
        for i, nm in enumerate(names):
            print("  %-14s %6.1f%%  %8.0f cyc/block" % (nm, 100 * R[:, i].sum() / tot, R[:, i].mean()))
        sym, stall, slow = P[:, 24].sum(), P[:, 25].sum(), P[:, 26].sum()
        print("  symbols/block %.0f, cycles/symbol %.1f, stalls/symbol %.3f, slow/symbol %.4f"
              % (sym / nb, tot / max(sym, 1), stall / max(sym, 1), slow / max(sym, 1)))
        print("  block cycles:", pct(R.sum(1)))
        # LZ77 pass (k_resolve): slots 2 total, 3 setup, 4 descriptors, 5 ordered rounds,
        # 12 pre matches, 13 write-back + slide; 6 rounds, 7 matches
        Q = P[:, [2, 3, 4, 12, 5, 13]]
        print("LZ77 pass, cycles per block (wave):")
        for i, nm in enumerate(["total", "setup", "descriptors", "pre matches", "ordered rounds",
                                "write-back+slide"]):
            print("  %-16s %s" % (nm, pct(Q[:, i])))
        print("  rounds/block %.0f, matches/block %.0f, cycles/round %.0f"
              % (P[:, 6].mean(), P[:, 7].mean(), P[:, 5].sum() / max(P[:, 6].sum(), 1)))
    else:
        L.hbam_prof_attach_guess.argtypes = [C.c_void_p]
        k = a.guesses
        pbuf = torch.zeros(k * 8, dtype=torch.int64, device="cuda")
        assert L.hbam_prof_attach_guess(C.c_void_p(pbuf.data_ptr())) == 0
        rng = np.random.default_rng(3)
        beg = np.sort(rng.integers(0, n - 1, k)).astype(np.int64)
        end = np.minimum(beg + (128 << 20), n).astype(np.int64)
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.time()
            rc, out, err = ctx.guess_batch(d[:n], beg, end, h["n_ref"])
            torch.cuda.synchronize()
            print("guess_batch %.3fs" % (time.time() - t0), flush=True)
            assert rc == 0
        P = pbuf.view(-1, 8).cpu().numpy().astype(np.float64)
        names = ["whole", "bgzf search", "bam search", "chain decode", "bgzf cands", "bam cands",
                 "records", "magics"]
        for i, nm in enumerate(names):
            print("  %-13s %s" % (nm, pct(P[:, i])))
        w = P[:, 0]
        top = np.argsort(w)[-20:]
        chk = np.unique(np.concatenate([top, [i for i in (4197, 7433) if i < k]])).astype(np.int64)
        for i in top[-5:]:
            print("  slow guess %d off %d:" % (i, beg[i]), P[i].astype(np.int64).tolist())
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        bad = 0
        for i in chk:  # the slowest guesses are the ones the chain memo short-cuts
            want = tuple(map(int, oracle.guess_bam_record_start(data, int(beg[i]), int(end[i]), h["n_ref"])))
            bad += (int(out[i]), int(err[i])) != want
        print("  oracle parity on the %d slowest guesses (+ r1's two slowest): %d mismatches" % (len(chk), bad), flush=True)


if __name__ == "__main__":
    main()
