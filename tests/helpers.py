"""Test helpers: derive the columnar pools the GPU emits from the oracle's raw variable
blocks (name | cigar | packed seq | qual | aux), so both sides compare field by field."""
import numpy as np

SEQ_ALPHA = np.frombuffer(b"=ACMGRSVTWYHKDBN", dtype=np.uint8)

FIELDS = ("voffset", "key", "block_size", "ref_id", "pos", "l_read_name", "mapq", "bin",
          "n_cigar", "flag", "l_seq", "next_ref_id", "next_pos", "tlen")


def oracle_pools(ref):
    n = ref["n"]
    names, cig, seq, qual, aux = [], [], [], [], []
    layout = np.zeros(n, np.uint8)
    for i in range(n):
        v = ref["var"][int(ref["var_off"][i]):int(ref["var_off"][i + 1])]
        L = int(ref["l_read_name"][i])
        nc = int(ref["n_cigar"][i])
        ls = int(ref["l_seq"][i])
        fixed = L + 4 * nc + (ls + 1) // 2 + ls
        if ls < 0 or fixed > len(v):
            continue
        layout[i] = 1
        p = 0
        names.append(v[p:p + L]); p += L
        cig.append(v[p:p + 4 * nc].view(np.uint32) if nc else np.zeros(0, np.uint32)); p += 4 * nc
        packed = v[p:p + (ls + 1) // 2]; p += (ls + 1) // 2
        hi = packed >> 4
        lo = packed & 15
        codes = np.empty(2 * len(packed), np.uint8)
        codes[0::2] = hi
        codes[1::2] = lo
        seq.append(SEQ_ALPHA[codes[:ls]])
        qual.append(v[p:p + ls]); p += ls
        aux.append(v[p:])
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return dict(layout_ok=layout, names=cat(names, np.uint8), cigars=cat(cig, np.uint32),
                seq=cat(seq, np.uint8), qual=cat(qual, np.uint8), aux=cat(aux, np.uint8))


def assert_same_split(got, ref, pools=True):
    assert got["n"] == ref["n"], (got["n"], ref["n"])
    assert got["status"] == ref["status"], (got["status"], ref["status"])
    if ref["status"] != 0:
        assert got["err_record"] == ref["err_record"]
    for k in FIELDS:
        assert np.array_equal(got[k], ref[k]), "column %s differs" % k
    if pools:
        op = oracle_pools(ref)
        assert np.array_equal(got["layout_ok"], op["layout_ok"])
        for k in ("names", "cigars", "seq", "qual", "aux"):
            assert np.array_equal(got[k], op[k]), "pool %s differs" % k
