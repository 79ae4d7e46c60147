"""Build the CPU model of the Huffman pass (tools/cpu_model/tok_model.cpp) under MemorySanitizer,
for the current source and for the round-2 source that failed in reused wave slots (commit
b49031e, DESIGN.md §4 "The r02 profiling-build decode failure").

The per-lane decode is compiled unchanged except for two substitutions that have no host
equivalent: the global-address-space quad pointer (a plain pointer on the host) and the packed
VOP3P lookup asm of `huffp_lookup` (restated in C below: per 16-bit half, g = (v + 1 > lim),
then the same accumulations the asm performs).  tools/cpu_model/hip/hip_runtime.h supplies the
few HIP names.  Diagnostic only; the product never links any of this.

usage: build.py OUTDIR [cur|r02|r02prof ...]   -> OUTDIR/tok_model_<variant>
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CLANG = os.environ.get("HBAM_MODEL_CXX", "/opt/rocm/lib/llvm/bin/clang++")
R02 = "b49031e"

LOOKUP_C = r'''template <bool HI>
__device__ __forceinline__ bool huffp_lookup(const HuffP& h, uint32_t v, uint32_t& L, uint32_t& idx,
                                             uint32_t& hi) {
  // CPU model of the packed sequence: per half q of pair j, g = min(sat(v + 1 - lim), 1)
  uint32_t sl = 0, so = 0, st = 0;
  for (int j = 0; j < 7; ++j) {
    for (int q = 0; q < 2; ++q) {
      const uint32_t lim = (h.lim[j] >> (16 * q)) & 0xffffu;
      const uint32_t g = (v + 1u > lim) ? 1u : 0u;
      const uint32_t dof = (h.dof[j] >> (16 * q)) & 0xffffu;
      const uint32_t dhl = HI ? ((h.dhl[j] >> (16 * q)) & 0xffffu) : 0u;
      sl += g;  // v_dot2_u32_u16 accumulation (both sources: the r02 one with HBAM_TOK_DOT2 = 1)
      so += g * dof;
      if (HI) st += g * dhl;
    }
  }
'''


def transform(src):
    """inflate_tok.h -> its host-model form (see the module docstring)."""
    out, n = re.subn(r"typedef const __attribute__\(\(address_space\(1\)\)\) u32x4_t\* gq_ptr;",
                     "typedef const u32x4_t* gq_ptr;", src)
    assert n == 1, "gq_ptr typedef not found"
    # the lookup: from its template line through the asm blocks up to the shared tail
    head = "template <bool HI>\n__device__ __forceinline__ bool huffp_lookup("
    i = out.index(head)
    # the shared tail: behind `#if HBAM_TOK_DOT2` in the r02 source, plain since round 5
    j = out.find("#if HBAM_TOK_DOT2\n  const uint32_t l = 1u + sl;", i)
    if j < 0:
        j = out.index("  const uint32_t l = 1u + sl;", i)
    return out[:i] + LOOKUP_C + out[j:]


def sources(variant, d):
    os.makedirs(d, exist_ok=True)
    if variant == "cur":
        tok = open(os.path.join(ROOT, "hadoop-bam_amd/csrc/inflate_tok.h")).read()
        dev = open(os.path.join(ROOT, "hadoop-bam_amd/csrc/inflate_dev.h")).read()
    else:
        show = lambda p: subprocess.run(["git", "-C", ROOT, "show", "%s:%s" % (R02, p)], check=True,
                                        stdout=subprocess.PIPE, text=True).stdout
        tok = show("hadoop-bam_amd/csrc/inflate_tok.h")
        dev = show("hadoop-bam_amd/csrc/inflate_dev.h")
    open(os.path.join(d, "inflate_tok.h"), "w").write(transform(tok))
    open(os.path.join(d, "inflate_dev.h"), "w").write(dev)


FLAGS = {"cur": [], "r02": ["-DHBAM_TOK_PRED=1"], "r02prof": ["-DHBAM_TOK_PRED=1", "-DHBAM_PROF"]}


def build(outdir, variant, sanitize=True, extra=(), tag=""):
    d = os.path.join(outdir, "src_" + variant)
    sources(variant, d)
    exe = os.path.join(outdir, "tok_model_" + variant + tag + ("" if sanitize else "_plain"))
    cmd = [CLANG, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fno-strict-aliasing",
           "-I", os.path.join(ROOT, "tools/cpu_model"), "-I", d] + FLAGS[variant] + list(extra)
    if sanitize:
        cmd += ["-fsanitize=memory", "-fsanitize-memory-track-origins=2"]
    cmd += ["-o", exe, os.path.join(ROOT, "tools/cpu_model/tok_model.cpp")]
    subprocess.run(cmd, check=True)
    return exe


if __name__ == "__main__":
    outdir = sys.argv[1]
    for v in sys.argv[2:] or ["cur", "r02", "r02prof"]:
        print(build(outdir, v))
