"""Build an A/B variant of libhbam.so with the product recipe (__graft_entry__.build: the Huffman
lane pass in its own max-ILP translation unit, everything else default-scheduled) plus extra
-D flags, into hadoop-bam_amd/NAME.  Never loaded by the tests, smoke() or bench.py unless
HBAM_LIB names it.
    python tools/ab_build.py libhbam_k8.so -DHBAM_TOK_K=8"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    # HBAM_AB_CAPI_FLAGS: extra flags for the hbam_capi.hip unit only (e.g. its own scheduler)
    capi_extra = os.environ.get("HBAM_AB_CAPI_FLAGS", "").split()
    obj = os.path.join(ROOT, "build", "ab", name)
    os.makedirs(obj, exist_ok=True)
    cflags = [f for f in g.HIP_FLAGS if f != "-shared"] + ["-c"] + defs
    o_tok, o_capi = os.path.join(obj, "tok.o"), os.path.join(obj, "capi.o")
    procs = [subprocess.Popen([g.HIPCC] + cflags + ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-o", o_tok,
                               os.path.join(g.CSRC, "hbam_inflate_tokens.hip")]),
             subprocess.Popen([g.HIPCC] + cflags + capi_extra + ["-DHBAM_SPLIT_TOK", "-o", o_capi,
                               os.path.join(g.CSRC, "hbam_capi.hip")])]
    if any(p.wait() for p in procs):
        sys.exit("ab_build: compile failed")
    subprocess.check_call([g.HIPCC, "-shared", "-fPIC", "--offload-arch=" + g.ARCH, "-o",
                           os.path.join(g.PKG, name), o_capi, o_tok])
    print("built hadoop-bam_amd/%s %s" % (name, " ".join(defs)))


if __name__ == "__main__":
    main()
