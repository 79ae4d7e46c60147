"""Synthetic BCF2 (v2.1) files for the BCF split-guesser tests: a VCF text
header (contigs, FILTER / INFO / FORMAT lines, samples) and records with typed values (BCF2
spec: l_shared, l_indiv, CHROM, POS, rlen, QUAL, n_allele_info, n_fmt_sample, ID, alleles,
FILTER, INFO, then the per-sample FORMAT block), BGZF-compressed by tests/helpers.bgzf_pack or
left uncompressed."""
import struct

import numpy as np

INT8, INT16, INT32, FLOAT, CHAR = 1, 2, 3, 5, 7


def typed_int(v):
    if -120 <= v <= 127:
        return bytes([0x10 | INT8]) + struct.pack("<b", v)
    if -32760 <= v <= 32767:
        return bytes([0x10 | INT16]) + struct.pack("<h", v)
    return bytes([0x10 | INT32]) + struct.pack("<i", v)


def typed_str(s):
    b = s.encode() if isinstance(s, str) else s
    if len(b) < 15:
        return bytes([(len(b) << 4) | CHAR]) + b
    return bytes([0xf0 | CHAR]) + typed_int(len(b)) + b


def typed_ints(vals, t=INT8):
    fmt = {INT8: "<b", INT16: "<h", INT32: "<i"}[t]
    head = bytes([(len(vals) << 4) | t]) if len(vals) < 15 else bytes([0xf0 | t]) + typed_int(len(vals))
    return head + b"".join(struct.pack(fmt, v) for v in vals)


def header_text(n_contig=25, samples=("S1", "S2", "S3")):
    lines = ["##fileformat=VCFv4.2", '##FILTER=<ID=PASS,Description="All filters passed">',
             '##FILTER=<ID=q10,Description="Quality below 10">',
             '##INFO=<ID=DP,Number=1,Type=Integer,Description="Depth">',
             '##INFO=<ID=AF,Number=A,Type=Float,Description="Allele frequency">',
             '##INFO=<ID=DB,Number=0,Type=Flag,Description="dbSNP">',
             '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">',
             '##FORMAT=<ID=DP,Number=1,Type=Integer,Description="Depth">']
    lines += ["##contig=<ID=chr%d,length=%d>" % (i + 1, 1000000 + i) for i in range(n_contig)]
    lines.append("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples))
    return "\n".join(lines) + "\n"


# the BCF2 string dictionary: PASS first, then FILTER / INFO / FORMAT IDs in header order
DICT = {"PASS": 0, "q10": 1, "DP": 2, "AF": 3, "DB": 4, "GT": 5}


def record(rng, chrom, pos, n_sample, long_id=False, hom_ref=0.0):
    bases = "ACGT"
    ref = "".join(rng.choice(list(bases), int(rng.integers(1, 4))))
    alts = ["".join(rng.choice(list(bases), int(rng.integers(1, 3)))) for _ in range(int(rng.integers(1, 3)))]
    rid = ("rs%d" % int(rng.integers(1, 10 ** 9))) * (3 if long_id else 1)
    info = [(DICT["DP"], typed_int(int(rng.integers(0, 300)))),
            (DICT["AF"], bytes([(len(alts) << 4) | FLOAT]) + b"".join(struct.pack("<f", float(rng.random())) for _ in alts))]
    if rng.random() < 0.3:
        info.append((DICT["DB"], bytes([0x00])))  # flag: a missing value
    shared = struct.pack("<iiif", chrom, pos, len(ref), float(rng.random() * 100))
    shared += struct.pack("<iI", (1 + len(alts)) << 16 | len(info), 2 << 24 | n_sample)
    shared += typed_str(rid)
    for a in [ref] + alts:
        shared += typed_str(a)
    shared += typed_ints([DICT["PASS"] if rng.random() < 0.8 else DICT["q10"]])
    for k, v in info:
        shared += typed_int(k) + v
    # hom_ref: share of samples with GT 0/0 and a typical depth (population VCFs compress 5-10x)
    ref = rng.random(n_sample) < hom_ref
    indiv = typed_int(DICT["GT"]) + bytes([(2 << 4) | INT8]) + b"".join(
        struct.pack("<bb", 2, 2) if r else
        struct.pack("<bb", int(rng.integers(1, 4)) * 2, int(rng.integers(1, 4)) * 2 | 1) for r in ref)
    indiv += typed_int(DICT["DP"]) + bytes([(1 << 4) | INT16]) + b"".join(
        struct.pack("<h", 30 if r else int(rng.integers(0, 500))) for r in ref)
    return struct.pack("<II", len(shared), len(indiv)) + shared + indiv


def bcf_stream(n_records=20000, seed=1, n_contig=25, samples=("S1", "S2", "S3"), hom_ref=0.0):
    """The uncompressed BCF2 stream: magic, l_text, the NUL-terminated header, records in
    coordinate order over the first few contigs."""
    rng = np.random.default_rng(seed)
    text = header_text(n_contig, samples).encode() + b"\0"
    out = [b"BCF\x02\x01", struct.pack("<I", len(text)), text]
    chrom, pos = 0, 100
    for i in range(n_records):
        pos += int(rng.integers(1, 400))
        if pos > 900000:
            chrom, pos = min(chrom + 1, n_contig - 1), 100
        out.append(record(rng, chrom, pos, len(samples), long_id=(i % 97 == 5), hom_ref=hom_ref))
    return b"".join(out)
