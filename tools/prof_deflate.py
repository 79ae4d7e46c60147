"""Where k_lz77_tokens spends its cycles (libhbam_prof.so, s_memtime of thread 0 per block):
whole block, match phase, barrier waits, greedy walk; walk iterations and tokens."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
os.environ["HBAM_LIB"] = os.path.join(ROOT, "hadoop-bam_amd", "libhbam_prof.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

g = genbam.generate(target_bytes=int(2e8), seed=5, threads=16)
data = np.asarray(g)
ctx = _lib.Context(0)
L = _lib.load()
rc, blocks = ctx.scan_blocks(data)
rc, u, off, st = ctx.inflate(data, blocks, check_crc=False)
src = torch.from_numpy(u).cuda()
nb = (len(u) + 65279) // 65280
pbuf = torch.zeros(8 * (nb + 8), dtype=torch.int64, device="cuda")
L.hbam_prof_attach_deflate.argtypes = [C.c_void_p]
assert L.hbam_prof_attach_deflate(C.c_void_p(pbuf.data_ptr())) == 0
ctx.bgzf_compress(src)
P = pbuf.view(-1, 8)[:min(nb, 4096)].cpu().numpy().astype(np.float64)
for i, nm in enumerate(["total", "walk", "sync", "walk iters", "tokens", "match"]):
    print("%-11s mean %12.0f p50 %12.0f max %12.0f" % (nm, P[:, i].mean(), np.median(P[:, i]), P[:, i].max()))
print("cycles per walk iteration %.1f" % (P[:, 1].sum() / max(P[:, 3].sum(), 1)))
