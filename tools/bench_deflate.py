"""BAM output throughput: the inflated stream of a synthetic BAM, resident
in HBM, compressed to BGZF by hbam_bgzf_compress (device source and destination); the result
is inflated back on the device and compared.  Ratio against the generator's zlib level 5
(htsjdk's default).  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=2e9, help="compressed bytes of the source BAM")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import genbam
    from hadoop_bam import _lib
    g = genbam.generate(target_bytes=int(a.size), seed=5, threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    data = np.asarray(g)
    ctx = _lib.Context(0)
    dcomp = torch.from_numpy(data).cuda()
    rc, blocks = ctx.scan_blocks(dcomp)
    assert rc == 0
    U = int(np.sum(blocks["isize"].astype(np.uint64)))
    src = torch.empty(U + 64, dtype=torch.uint8, device="cuda")
    rc, u, off, st = ctx.inflate(dcomp, blocks, check_crc=False)  # host copy of the stream
    src[:U].copy_(torch.from_numpy(u[:U]))
    del u
    out = torch.empty(int(ctx.L.hbam_bgzf_bound(U, 0)), dtype=torch.uint8, device="cuda")
    times = []
    n = 0
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t = time.time()
        n = ctx.bgzf_compress(src[:U], 0, out=out)
        torch.cuda.synchronize()
        if r:
            times.append(time.time() - t)
    dev_ms = ctx.timing()["total_ms"]
    rc, b2 = ctx.scan_blocks(out[:n])
    assert rc == 0
    rc, u2, off2, st2 = ctx.inflate(out[:n], b2, check_crc=True)
    ok = rc == 0 and bool(np.all(st2 == 0)) and len(u2) == U and \
        bool(torch.equal(torch.from_numpy(u2[:U]).cuda(), src[:U]))
    best = min(times)
    print(json.dumps({
        "metric": "BGZF compress (BAM output, device deflate, one MI355X)", "value": round(U / best / 1e9, 3),
        "unit": "GB/s uncompressed", "uncompressed_bytes": U, "compressed_bytes": int(n),
        "ratio": round(U / n, 3), "zlib5_ratio": round(U / len(data), 3), "seconds": round(best, 4),
        "device_ms_last": round(dev_ms, 2), "blocks": int(len(b2["coff"])),
        "inflates_back_crc_checked": ok}), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
