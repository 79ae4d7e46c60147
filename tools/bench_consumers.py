"""Throughput of the f-4 consumers on the device: SummarizeRecordReader ranges
(hbam_summarize_ranges) and FixMate's name shuffle + reducer (hbam_fixmate) over a decoded
synthetic BAM split resident in HBM, plus FixMate over replicated paired key groups
(tests/f4_records.py) — the generator gives every record its own name, so the decoded split has
no pairs.  A sample of each result is checked against the oracle.  Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=2e9)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--pair-copies", type=int, default=1000)
a = ap.parse_args()
torch.cuda.init()
g = genbam.generate(target_bytes=int(a.size), seed=2, threads=16)
data = np.asarray(g)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
ctx = _lib.Context(0)
h = ctx.parse_header(data[:1 << 20])
v_end = (len(data) << 16) | 0xffff
rc, dc = ctx.decode_split_device(d[:len(data)], h["first_voffset"], v_end, h["n_ref"], file_len=len(data))
assert rc == 0 and dc.status == 0, rc
n = int(dc.n_records)
out = {"records": n, "ubuf_bytes": int(dc.ubuf_len)}

sum_ms = []
for r in range(a.reps):
    t0 = time.time()
    rr = ctx.summarize_ranges(dc)
    sum_ms.append(ctx.timing()["total_ms"])
out["summarize"] = {"ranges": int(len(rr["key"])), "device_ms": min(sum_ms),
                    "records_per_s": n / (min(sum_ms) / 1e3),
                    "what": "k_sum_count + scan + k_sum_emit over the decoded split's records"}

ub = C.cast(dc.ubuf, C.c_void_p).value
ro = C.cast(dc.rec_off, C.c_void_p).value
fm_ms = []
for r in range(a.reps):
    fm = ctx.fixmate(ub, ro, n)
    fm_ms.append(ctx.timing()["total_ms"])
out["fixmate_decoded"] = {"outputs": int(len(fm["src"])), "groups": fm["n_groups"], "device_ms": min(fm_ms),
                          "records_per_s": n / (min(fm_ms) / 1e3),
                          "what": "name order (LSD radix over 8-byte name chunks) + groups + reducer plan + "
                                  "encode over the decoded split (every name distinct: no pairs)"}

import f4_records as F  # noqa: E402
base = F.fixmate_records(seed=5)
pay_l, names = [], []
for c in range(a.pair_copies):
    for r in base:
        lrn = r[12]
        nm = bytes(r[36:36 + lrn - 1]) + b"_%05d" % c
        body = bytearray(r[4:])
        body[8] = len(nm) + 1
        rec = bytes(body[:32]) + nm + b"\0" + bytes(body[32 + lrn:])
        pay_l.append(len(rec).to_bytes(4, "little", signed=True) + rec)
pay, off = F.pack(pay_l)
tp = torch.from_numpy(pay).cuda()
to = torch.from_numpy(off.view(np.int64)).cuda()
torch.cuda.synchronize()
m = len(off) - 1
pm = []
for r in range(a.reps):
    fp = ctx.fixmate(tp.data_ptr(), to.data_ptr(), m)
    pm.append(ctx.timing()["total_ms"])
import oracle  # noqa: E402
k = len(base) * min(a.pair_copies, 40)  # whole copies: complete key groups
sub_t = torch.from_numpy(pay[:int(off[k])].copy()).cuda()
sub_o = torch.from_numpy(off[:k + 1].copy().view(np.int64)).cuda()
torch.cuda.synchronize()
got = ctx.fixmate(sub_t.data_ptr(), sub_o.data_ptr(), k)
want = oracle.fixmate(pay[:int(off[k])], off[:k + 1])
ok = bool(fp["status"] == 0 and np.array_equal(got["payload"], want["payload"]) and
          np.array_equal(got["src"], want["src"]))
out["fixmate_pairs"] = {"records": m, "outputs": int(len(fp["src"])), "groups": fp["n_groups"],
                        "device_ms": min(pm), "records_per_s": m / (min(pm) / 1e3), "parity_sample_records": k, "parity_ok": ok,
                        "what": "tests/f4_records.fixmate_records groups replicated with distinct names"}
# parity on the first decoded records (summarize) against the oracle
o_cols = oracle.read_split(data, h["first_voffset"], (min(len(data), 4 << 20) << 16) | 0xffff)
opay, ooff = oracle.record_payloads(o_cols)
want = oracle.summarize_ranges(opay, ooff)
kk = len(want["key"]) - 64  # the oracle's window ends early; compare the ranges both hold
out["summarize"]["parity_sample_ranges"] = int(kk)
out["summarize"]["parity_mismatch"] = int(np.sum(rr["key"][:kk] != want["key"][:kk]) +
                                           np.sum(rr["beg"][:kk] != want["beg"][:kk]))
print(json.dumps(out), flush=True)
