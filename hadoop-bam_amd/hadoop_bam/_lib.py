"""ctypes binding of libhbam.so (include/hbam.h).

The product path is the HIP library only: if libhbam.so is missing or cannot create a
device context, calls raise HbamUnavailable — there is no CPU fallback.
"""
import ctypes as C
import sys
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # hadoop-bam_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.path.join(PKG_ROOT, "libhbam.so")

HBAM_OK = 0
HBAM_EIO = -1
HBAM_ETRUNC = -2
HBAM_EFORMAT = -3
HBAM_ERUNTIMEIO = -4
HBAM_EEOF = -5
HBAM_EREFID = -6
HBAM_EDATA = -7
HBAM_ENOMEM = -8
HBAM_EUNSUPPORTED = -9
HBAM_EDEVICE = -10
HBAM_EINVAL = -11
HBAM_EMORE = -12
HBAM_EINDEX = -13
HBAM_ETRIBBLE = -14
HBAM_ERUNTIME = -15
HBAM_ENULL = -16
HBAM_ECLASSCAST = -17

CODE_NAMES = {
    HBAM_OK: "OK", HBAM_EIO: "IOException", HBAM_ETRUNC: "FileTruncatedException",
    HBAM_EFORMAT: "SAMFormatException", HBAM_ERUNTIMEIO: "RuntimeIOException",
    HBAM_EEOF: "RuntimeEOFException", HBAM_EREFID: "IllegalArgumentException",
    HBAM_EDATA: "RuntimeException(DataFormatException)", HBAM_ENOMEM: "OutOfMemory",
    HBAM_EUNSUPPORTED: "Unsupported", HBAM_EDEVICE: "DeviceError", HBAM_EINVAL: "InvalidArgument",
    HBAM_EMORE: "NeedMoreData", HBAM_EINDEX: "IndexOutOfBoundsException",
    HBAM_ETRIBBLE: "TribbleException", HBAM_ERUNTIME: "RuntimeException",
    HBAM_ENULL: "NullPointerException", HBAM_ECLASSCAST: "ClassCastException",
}

# every entry point include/hbam.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "hbam_create", "hbam_destroy", "hbam_last_error", "hbam_stream", "hbam_get_timing",
    "hbam_upload", "hbam_device_free", "hbam_parse_header", "hbam_scan_blocks", "hbam_inflate",
    "hbam_decode_split", "hbam_columns_to_host", "hbam_free_host_columns",
    "hbam_release_columns", "hbam_guess_bam_record_start", "hbam_guess_batch",
    "hbam_guess_bgzf_block_start", "hbam_probabilistic_splits",
    "hbam_sort_keys", "hbam_gather_records", "hbam_permute", "hbam_splitting_index",
    "hbam_bgzf_block_index", "hbam_resolve_tokens", "hbam_split_open", "hbam_split_next",
    "hbam_split_stats", "hbam_split_close", "hbam_device_alloc", "hbam_sort_split",
    "hbam_sort_partition", "hbam_sort_received", "hbam_bgzf_bound", "hbam_bgzf_compress",
    "hbam_summarize_ranges", "hbam_name_order", "hbam_fixmate", "hbam_download",
    "hbam_guess_window_len", "hbam_guess_windows", "hbam_guess_bgzf_window_len",
    "hbam_guess_bgzf_window", "hbam_probabilistic_splits_windows", "hbam_merge_remap",
    "hbam_host_register", "hbam_host_unregister", "hbam_bcf_parse_header", "hbam_guess_bcf_window_len",
    "hbam_guess_bcf_windows", "hbam_bcf_decode_split", "hbam_comm_unique_id", "hbam_comm_init",
    "hbam_comm_destroy", "hbam_comm_split_points", "hbam_sort_exchange", "hbam_split_open_reader",
    "hbam_split_read_bytes", "hbam_rewrite_groups", "hbam_records_to_host", "hbam_split_records_to_host",
]

# hbam_read_fn: int64_t read(void* user, uint64_t offset, uint64_t len, uint8_t* dst)
READ_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p)


class HbamUnavailable(RuntimeError):
    pass


class Opts(C.Structure):
    _fields_ = [("check_crc", C.c_int32), ("validate_refs", C.c_int32),
                ("reserved", C.c_int32 * 14)]


class Header(C.Structure):
    _fields_ = [("l_text", C.c_int32), ("n_ref", C.c_int32), ("header_ulen", C.c_uint64),
                ("first_voffset", C.c_uint64)]


class Block(C.Structure):
    _fields_ = [("coff", C.c_uint64), ("clen", C.c_uint32), ("isize", C.c_uint32),
                ("crc", C.c_uint32), ("pad", C.c_uint32)]


class Timing(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("scan_ms", "inflate_ms", "crc_ms", "walk_ms",
                                          "decode_ms", "pools_ms", "total_ms",
                                          "huffman_ms", "resolve_ms")] + \
               [(n, C.c_uint64) for n in ("n_blocks", "comp_bytes", "ubuf_bytes", "n_records",
                                          "pool_bytes")] + [("exchange_ms", C.c_double)]


class SortedRunC(C.Structure):
    _fields_ = [("n", C.c_uint64), ("payload_bytes", C.c_uint64), ("key", C.c_void_p),
                ("voffset", C.c_void_p), ("block_size", C.c_void_p), ("offsets", C.c_void_p),
                ("payload", C.c_void_p)]


class RangesC(C.Structure):
    _fields_ = [("n", C.c_uint64), ("status", C.c_int32), ("pad", C.c_int32), ("key", C.c_void_p),
                ("beg", C.c_void_p), ("end", C.c_void_p), ("rev", C.c_void_p), ("record", C.c_void_p)]


class FixmateRunC(C.Structure):
    _fields_ = [("n", C.c_uint64), ("payload_bytes", C.c_uint64), ("n_groups", C.c_uint64),
                ("status", C.c_int32), ("pad", C.c_int32), ("src", C.c_void_p), ("mate", C.c_void_p),
                ("offsets", C.c_void_p), ("payload", C.c_void_p)]


class BcfHeaderC(C.Structure):
    _fields_ = [("n_contig", C.c_int32), ("n_sample", C.c_int32), ("n_dict", C.c_int32),
                ("bgzf", C.c_int32), ("header_len", C.c_uint64), ("first_voffset", C.c_uint64)]


_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class Columns(C.Structure):
    _fields_ = [
        ("n_records", C.c_uint64), ("status", C.c_int32), ("pad0", C.c_int32),
        ("err_record", C.c_uint64), ("voffset", _u64p), ("key", _i64p), ("rec_off", _u64p),
        ("ubuf", _u8p), ("ubuf_len", C.c_uint64), ("block_size", _i32p), ("ref_id", _i32p),
        ("pos", _i32p), ("l_read_name", _u8p), ("mapq", _u8p), ("bin", _u16p),
        ("n_cigar", _u16p), ("flag", _u16p), ("l_seq", _i32p), ("next_ref_id", _i32p),
        ("next_pos", _i32p), ("tlen", _i32p), ("layout_ok", _u8p), ("name_off", _u64p),
        ("names", _u8p), ("cigar_off", _u64p), ("cigars", _u32p), ("seq_off", _u64p),
        ("seq", _u8p), ("qual", _u8p), ("aux_off", _u64p), ("aux", _u8p),
    ]


class BcfColumnsC(C.Structure):
    _fields_ = [
        ("n_records", C.c_uint64), ("status", C.c_int32), ("pad0", C.c_int32),
        ("err_record", C.c_uint64), ("rel", C.c_void_p), ("rec_off", C.c_void_p), ("data", C.c_void_p),
        ("data_len", C.c_uint64), ("key", C.c_void_p), ("l_shared", C.c_void_p), ("l_indiv", C.c_void_p),
        ("chrom", C.c_void_p), ("pos", C.c_void_p), ("rlen", C.c_void_p), ("qual", C.c_void_p),
        ("n_allele_info", C.c_void_p), ("n_fmt_sample", C.c_void_p),
    ]


BCF_FIELDS = [("rel", np.int64), ("rec_off", np.uint64), ("key", np.int64), ("l_shared", np.int32),
              ("l_indiv", np.int32), ("chrom", np.int32), ("pos", np.int32), ("rlen", np.int32),
              ("qual", np.uint32), ("n_allele_info", np.int32), ("n_fmt_sample", np.int32)]


FIXED = [("voffset", np.uint64), ("key", np.int64), ("rec_off", np.uint64),
         ("block_size", np.int32), ("ref_id", np.int32), ("pos", np.int32),
         ("l_read_name", np.uint8), ("mapq", np.uint8), ("bin", np.uint16),
         ("n_cigar", np.uint16), ("flag", np.uint16), ("l_seq", np.int32),
         ("next_ref_id", np.int32), ("next_pos", np.int32), ("tlen", np.int32),
         ("layout_ok", np.uint8)]

_LIB = None


def load(path=None):
    """Load libhbam.so (raises HbamUnavailable if it is not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("HBAM_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise HbamUnavailable("libhbam.so not built (run __graft_entry__.build())")
    L = C.CDLL(path)
    vp = C.c_void_p
    sig = {
        "hbam_create": (vp, [C.c_int, C.POINTER(Opts)]),
        "hbam_destroy": (None, [vp]),
        "hbam_last_error": (C.c_char_p, [vp]),
        "hbam_stream": (vp, [vp]),
        "hbam_get_timing": (C.c_int, [vp, C.POINTER(Timing)]),
        "hbam_upload": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(vp)]),
        "hbam_device_free": (C.c_int, [vp, vp]),
        "hbam_download": (C.c_int, [vp, vp, C.c_uint64, vp]),
        "hbam_parse_header": (C.c_int, [vp, vp, C.c_int, C.c_uint64, C.POINTER(Header)]),
        "hbam_scan_blocks": (C.c_int, [vp, vp, C.c_int, C.c_uint64, C.c_uint64,
                                       C.POINTER(Block), C.c_uint64, C.POINTER(C.c_uint64)]),
        "hbam_inflate": (C.c_int, [vp, vp, C.c_int, C.c_uint64, C.POINTER(Block), C.c_uint64,
                                   C.c_int, vp, C.c_uint64, vp, vp]),
        "hbam_decode_split": (C.c_int, [vp, vp, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                        C.c_uint64, C.c_uint64, C.c_int32, C.POINTER(Columns)]),
        "hbam_columns_to_host": (C.c_int, [vp, C.POINTER(Columns), C.POINTER(Columns)]),
        "hbam_free_host_columns": (None, [C.POINTER(Columns)]),
        "hbam_records_to_host": (C.c_int, [vp, C.POINTER(Columns), C.POINTER(Columns)]),
        "hbam_split_records_to_host": (C.c_int, [vp, C.POINTER(Columns), C.POINTER(Columns)]),
        "hbam_release_columns": (None, [vp, C.POINTER(Columns)]),
        "hbam_guess_bam_record_start": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, C.c_int64,
                                                    C.c_int64, C.c_int32, _i32p]),
        "hbam_guess_batch": (C.c_int, [vp, vp, C.c_int, C.c_uint64, vp, vp, C.c_uint64,
                                       C.c_int32, vp, vp]),
        "hbam_guess_bgzf_block_start": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, C.c_int64,
                                                    C.c_int64, _i32p]),
        "hbam_probabilistic_splits": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, vp, vp,
                                                  C.c_uint64, vp, vp]),
        "hbam_guess_window_len": (C.c_uint64, [C.c_uint64, C.c_int64, C.c_int64]),
        "hbam_guess_bgzf_window_len": (C.c_uint64, [C.c_uint64, C.c_int64, C.c_int64]),
        "hbam_guess_windows": (C.c_int, [vp, vp, C.c_int, vp, C.c_uint64, vp, vp, C.c_uint64,
                                         C.c_int32, vp, vp]),
        "hbam_guess_bgzf_window": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, C.c_uint64, C.c_int64,
                                               C.c_int64, _i32p]),
        "hbam_probabilistic_splits_windows": (C.c_int64, [vp, vp, C.c_uint64, vp, C.c_int, vp,
                                                          C.c_uint64, vp, vp, C.c_uint64, vp, vp]),
        "hbam_sort_keys": (C.c_int, [vp, vp, C.c_uint64, vp, vp]),
        "hbam_gather_records": (C.c_int, [vp, vp, vp, vp, vp, C.c_uint64, vp, C.c_uint64, vp,
                                          C.POINTER(C.c_uint64)]),
        "hbam_permute": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint64, vp]),
        "hbam_splitting_index": (C.c_int64, [vp, C.POINTER(Columns), C.c_int32, C.c_uint64, vp,
                                             C.c_uint64]),
        "hbam_bgzf_block_index": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, C.c_int32, vp,
                                              C.c_uint64]),
        "hbam_resolve_tokens": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32, C.c_uint32, _i32p]),
        "hbam_split_open": (vp, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64]),
        "hbam_split_next": (C.c_int, [vp, C.POINTER(Columns)]),
        "hbam_split_open_reader": (vp, [vp, READ_FN, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32,
                                        C.c_uint64]),
        "hbam_split_read_bytes": (C.c_uint64, [vp]),
        "hbam_rewrite_groups": (C.c_int, [vp, C.POINTER(Columns), vp, C.c_uint64, _i32p, C.POINTER(C.c_uint64)]),
        "hbam_split_stats": (C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_double),
                                       C.POINTER(C.c_uint64)]),
        "hbam_split_close": (None, [vp]),
        "hbam_device_alloc": (C.c_int, [vp, C.c_uint64, C.POINTER(vp)]),
        "hbam_sort_split": (C.c_int, [vp, C.POINTER(Columns), C.POINTER(SortedRunC)]),
        "hbam_sort_partition": (C.c_int, [vp, C.POINTER(SortedRunC), vp, C.c_uint32, vp, vp]),
        "hbam_sort_received": (C.c_int, [vp, vp, vp, vp, vp, C.c_uint64, C.POINTER(SortedRunC)]),
        "hbam_merge_remap": (C.c_int, [vp, C.POINTER(Columns), vp, C.c_int32, C.POINTER(C.c_uint64)]),
        "hbam_host_register": (C.c_int, [vp, vp, C.c_uint64]),
        "hbam_host_unregister": (C.c_int, [vp, vp]),
        "hbam_bgzf_bound": (C.c_uint64, [C.c_uint64, C.c_uint32]),
        "hbam_bcf_parse_header": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(BcfHeaderC)]),
        "hbam_guess_bcf_window_len": (C.c_uint64, [C.c_uint64, C.c_int64, C.c_int64, C.c_int]),
        "hbam_guess_bcf_windows": (C.c_int, [vp, vp, C.c_int, vp, C.c_uint64, vp, vp, C.c_uint64,
                                             C.POINTER(BcfHeaderC), vp, vp]),
        "hbam_bcf_decode_split": (C.c_int, [vp, vp, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                            C.POINTER(BcfHeaderC), C.c_uint64, C.c_uint64,
                                            C.POINTER(BcfColumnsC)]),
        "hbam_summarize_ranges": (C.c_int, [vp, C.POINTER(Columns), C.POINTER(RangesC)]),
        "hbam_name_order": (C.c_int, [vp, vp, vp, C.c_uint64, vp]),
        "hbam_fixmate": (C.c_int, [vp, vp, vp, C.c_uint64, C.POINTER(FixmateRunC)]),
        "hbam_bgzf_compress": (C.c_int64, [vp, vp, C.c_int, C.c_uint64, C.c_uint32, vp, C.c_int,
                                           C.c_uint64]),
        "hbam_comm_unique_id": (C.c_int, [vp]),
        "hbam_comm_init": (C.c_int, [vp, vp, C.c_int32, C.c_int32, C.POINTER(vp)]),
        "hbam_comm_destroy": (None, [vp]),
        "hbam_comm_split_points": (C.c_int, [vp, vp, C.POINTER(SortedRunC), C.c_uint32, vp]),
        "hbam_sort_exchange": (C.c_int, [vp, vp, C.POINTER(SortedRunC), vp, C.POINTER(SortedRunC)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None:  # an older build (A/B runs): only what it exports is bound
            continue
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def host_columns_to_numpy(h):
    """Copy a host hbam_columns into a dict of numpy arrays."""
    n = int(h.n_records)
    out = {"n": n, "status": int(h.status), "err_record": int(h.err_record)}
    for name, dt in FIXED:
        p = getattr(h, name)
        out[name] = np.ctypeslib.as_array(p, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)
    for name in ("name_off", "cigar_off", "seq_off", "aux_off"):
        p = getattr(h, name)
        out[name] = np.ctypeslib.as_array(p, shape=(n + 1,)).copy() if p else np.zeros(1, np.uint64)
    ul = int(h.ubuf_len)
    out["ubuf"] = np.ctypeslib.as_array(h.ubuf, shape=(ul,)).copy() if (ul and h.ubuf) else np.zeros(0, np.uint8)
    pools = [("names", np.uint8, "name_off"), ("cigars", np.uint32, "cigar_off"),
             ("seq", np.uint8, "seq_off"), ("qual", np.uint8, "seq_off"),
             ("aux", np.uint8, "aux_off")]
    for name, dt, off in pools:
        m = int(out[off][-1]) if n else 0
        p = getattr(h, name)
        out[name] = np.ctypeslib.as_array(p, shape=(m,)).astype(dt).copy() if m else np.zeros(0, dt)
    return out


class Context:
    """One device context (hbam_ctx): a HIP stream plus device work buffers."""

    def __init__(self, device=0, check_crc=False, validate_refs=True):
        self.L = load()
        # PyTorch-ROCm ships its own HIP runtime; when both live in one process, torch's must
        # open the device first (the other order leaves torch with "No HIP GPUs").
        if "torch" in sys.modules:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        o = Opts()
        o.check_crc = int(check_crc)
        o.validate_refs = int(validate_refs)
        self.h = self.L.hbam_create(device, C.byref(o))
        if not self.h:
            raise HbamUnavailable("hbam_create failed: no HIP device %d" % device)

    def close(self):
        if getattr(self, "h", None):
            self.L.hbam_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self):
        return self.L.hbam_last_error(self.h).decode(errors="replace")

    def timing(self):
        t = Timing()
        self.L.hbam_get_timing(self.h, C.byref(t))
        return {n: getattr(t, n) for n, _ in Timing._fields_}

    @staticmethod
    def _ptr(data, output=False):
        """(pointer, length, on_device, keepalive) for bytes / numpy / torch cuda tensor.  An
        output buffer (the library writes into it) is never replaced by a padded copy."""
        if hasattr(data, "data_ptr") and hasattr(data, "is_cuda"):
            if data.is_cuda:
                # libhbam reads the raw pointer on its own stream: the bytes must be one dense
                # run, and whatever torch is still producing into them (a torch.cat, a .to(dev),
                # an all_to_all) must be finished first
                if not data.is_contiguous():
                    raise ValueError("device input must be contiguous")
                import torch
                nbytes = data.numel() * data.element_size()
                # the kernels read whole 16-byte quads and fixed windows past the last byte: 64
                # readable bytes must follow (include/hbam.h); a view that ends at (or near) the end
                # of its allocation is copied into a padded buffer first
                room = data.untyped_storage().nbytes() - data.storage_offset() * data.element_size()
                if room < nbytes + 64 and not output:
                    pad = torch.zeros(nbytes + 64, dtype=torch.uint8, device=data.device)
                    pad[:nbytes].copy_(data.reshape(-1).view(torch.uint8))
                    data = pad
                torch.cuda.current_stream(data.device).synchronize()
                return C.c_void_p(data.data_ptr()), nbytes, 1, data
            a = data.numpy()
        elif isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data, dtype=np.uint8)
        else:
            a = np.frombuffer(bytes(data), dtype=np.uint8)
        if a.size == 0:
            a = np.zeros(1, np.uint8)
            return C.c_void_p(a.ctypes.data), 0, 0, a
        return C.c_void_p(a.ctypes.data), a.size, 0, a

    def bgzf_compress(self, data, block_size=0, out=None):
        """BlockCompressedOutputStream over `data` (bytes / numpy / torch tensor, host or device)
        with the device deflate (hbam_bgzf_compress): the BGZF members, no terminator.  Returns
        a numpy uint8 array, or writes into the device tensor `out` and returns its length."""
        p, n, dev, keep = self._ptr(data)
        bound = int(self.L.hbam_bgzf_bound(n, block_size))
        if out is not None:
            q, cap, odev, okeep = self._ptr(out, output=True)
            r = self.L.hbam_bgzf_compress(self.h, p, dev, n, block_size, q, odev, cap)
            if r < 0:
                raise RuntimeError("hbam_bgzf_compress failed (%d): %s" % (r, self.last_error()))
            return int(r)
        buf = np.empty(max(bound, 1), np.uint8)
        r = self.L.hbam_bgzf_compress(self.h, p, dev, n, block_size, C.c_void_p(buf.ctypes.data), 0, bound)
        if r < 0:
            raise RuntimeError("hbam_bgzf_compress failed (%d): %s" % (r, self.last_error()))
        return buf[:r]

    def parse_header(self, data):
        p, n, dev, keep = self._ptr(data)
        h = Header()
        rc = self.L.hbam_parse_header(self.h, p, dev, n, C.byref(h))
        if rc:
            return rc
        return dict(l_text=h.l_text, n_ref=h.n_ref, header_ulen=h.header_ulen,
                    first_voffset=h.first_voffset)

    def scan_blocks(self, data, base_off=0):
        p, n, dev, keep = self._ptr(data)
        cap = n // 18 + 2
        arr = (Block * cap)()
        nb = C.c_uint64(0)
        rc = self.L.hbam_scan_blocks(self.h, p, dev, n, base_off, arr, cap, C.byref(nb))
        k = int(nb.value)
        out = dict(coff=np.array([arr[i].coff for i in range(k)], np.uint64),
                   clen=np.array([arr[i].clen for i in range(k)], np.uint32),
                   isize=np.array([arr[i].isize for i in range(k)], np.uint32),
                   crc=np.array([arr[i].crc for i in range(k)], np.uint32))
        return rc, out

    def inflate(self, data, blocks, check_crc=True):
        p, n, dev, keep = self._ptr(data)
        k = len(blocks["coff"])
        arr = (Block * max(k, 1))()
        for i in range(k):
            arr[i].coff = int(blocks["coff"][i])
            arr[i].clen = int(blocks["clen"][i])
            arr[i].isize = int(blocks["isize"][i])
            arr[i].crc = int(blocks["crc"][i])
        total = int(np.sum(blocks["isize"], dtype=np.uint64)) if k else 0
        out = np.zeros(max(total, 1), np.uint8)
        off = np.zeros(k + 1, np.uint64)
        st = np.zeros(max(k, 1), np.int32)
        rc = self.L.hbam_inflate(self.h, p, dev, n, arr, k, int(check_crc),
                                 out.ctypes.data, out.size, off.ctypes.data, st.ctypes.data)
        return rc, out[:total], off, st[:k]

    def decode_split(self, data, v_start, v_end, n_ref=-1, comp_base=0, file_len=None):
        """BAMRecordReader over one FileVirtualSplit; returns host numpy columns."""
        p, n, dev, keep = self._ptr(data)
        if file_len is None:
            file_len = comp_base + n
        d = Columns()
        rc = self.L.hbam_decode_split(self.h, p, dev, comp_base, n, file_len, v_start, v_end,
                                      n_ref, C.byref(d))
        if rc:
            return {"rc": rc, "error": self.last_error()}
        h = Columns()
        rc = self.L.hbam_columns_to_host(self.h, C.byref(d), C.byref(h))
        if rc:
            return {"rc": rc, "error": self.last_error()}
        out = host_columns_to_numpy(h)
        self.L.hbam_free_host_columns(C.byref(h))
        out["rc"] = 0
        out["timing"] = self.timing()
        return out

    def split_stream(self, data, v_start, v_end, n_ref, window_bytes=1 << 30, host=True):
        """Streamed BAMRecordReader over a host-resident file (hbam_split_open/next): yields
        the host columns of each window in order; the last one carries the split's status.
        host=False yields each window's device Columns struct instead (valid until the next
        window is requested); host="records" the records-only copy (records_to_host: views, valid
        until the next window is requested)."""
        a = np.ascontiguousarray(np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray)
                                 else data, dtype=np.uint8)
        keep = a if a.size else np.zeros(1, np.uint8)
        s = self.L.hbam_split_open(self.h, C.c_void_p(keep.ctypes.data), a.size, v_start, v_end,
                                   int(n_ref), int(window_bytes))
        if not s:
            raise HbamUnavailable("hbam_split_open failed: %s" % self.last_error())
        return self._stream(s, host, keep)

    def split_stream_reader(self, read, file_len, v_start, v_end, n_ref, window_bytes=1 << 30, host=True):
        """Split-local streamed BAMRecordReader (hbam_split_open_reader): read(offset, length) ->
        bytes is a positioned read of the file (os.pread, FSDataInputStream.read(long, ...)); only
        the blocks the split needs are requested.  Yields as split_stream."""
        def cb(user, off, n, dst):
            b = read(int(off), int(n))
            if not b:
                return -1
            if len(b) > n:  # never past the n bytes of staging the library asked to fill
                b = b[:n]
            C.memmove(dst, bytes(b), len(b))
            return len(b)
        fn = READ_FN(cb)
        s = self.L.hbam_split_open_reader(self.h, fn, None, int(file_len), v_start, v_end, int(n_ref),
                                          int(window_bytes))
        if not s:
            raise HbamUnavailable("hbam_split_open_reader failed: %s" % self.last_error())
        return self._stream(s, host, fn)

    def _stream(self, s, host, keep):
        try:
            while True:
                d = Columns()
                rc = self.L.hbam_split_next(s, C.byref(d))
                if rc < 0:
                    raise RuntimeError("hbam_split_next failed (%d): %s" % (rc, self.last_error()))
                if rc == 0:
                    return
                if not host:
                    yield d
                    continue
                if host == "records":
                    yield self.records_to_host(d, stream=s)
                    continue
                h = Columns()
                rc = self.L.hbam_columns_to_host(self.h, C.byref(d), C.byref(h))
                if rc:
                    raise RuntimeError("hbam_columns_to_host failed (%d): %s" % (rc, self.last_error()))
                out = host_columns_to_numpy(h)
                self.L.hbam_free_host_columns(C.byref(h))
                yield out
        finally:
            self.last_stream_stats = self._split_stats(s)
            self.L.hbam_split_close(s)
            del keep

    def records_to_host(self, d, stream=None):
        """hbam_records_to_host: what the drop-in reader hands out (key, voffset, rec_off, block_size
        and the records' bytes), as numpy VIEWS of the context's pinned staging — valid until the
        next call on this context; with `stream` (a split stream handle) hbam_split_records_to_host,
        views of that stream's own staging, valid until its next window or close whatever other
        readers of the context do.  d2h_bytes = what crossed PCIe."""
        h = Columns()
        if stream is not None:
            rc = self.L.hbam_split_records_to_host(stream, C.byref(d), C.byref(h))
        else:
            rc = self.L.hbam_records_to_host(self.h, C.byref(d), C.byref(h))
        if rc:
            raise RuntimeError("hbam_records_to_host failed (%d): %s" % (rc, self.last_error()))
        n = int(h.n_records)
        out = {"n": n, "status": int(h.status), "err_record": int(h.err_record)}
        for name, dt in (("voffset", np.uint64), ("key", np.int64), ("rec_off", np.uint64),
                         ("block_size", np.int32)):
            p = getattr(h, name)
            out[name] = np.ctypeslib.as_array(p, shape=(n,)).view(dt) if n else np.zeros(0, dt)
        ul = int(h.ubuf_len)
        out["ubuf"] = np.ctypeslib.as_array(h.ubuf, shape=(ul,)) if (ul and h.ubuf) else np.zeros(0, np.uint8)
        out["d2h_bytes"] = 28 * n + ul
        return out

    def _split_stats(self, s):
        b, w = C.c_uint64(0), C.c_uint64(0)
        ms = C.c_double(0)
        self.L.hbam_split_stats(s, C.byref(b), C.byref(ms), C.byref(w))
        return {"h2d_bytes": int(b.value), "h2d_ms": float(ms.value), "windows": int(w.value),
                "read_bytes": int(self.L.hbam_split_read_bytes(s))}

    def download(self, ptr, nbytes, dtype=np.uint8):
        """hbam_download: `nbytes` of device memory at address `ptr` -> numpy array of dtype."""
        a = np.empty(max(int(nbytes), 1), np.uint8)
        if nbytes:
            rc = self.L.hbam_download(self.h, C.c_void_p(int(ptr)), int(nbytes), C.c_void_p(a.ctypes.data))
            if rc:
                raise RuntimeError("hbam_download failed (%d): %s" % (rc, self.last_error()))
        return a[:int(nbytes)].view(dtype)

    def columns_slice(self, d, i0, i1):
        """Host copy of records [i0, i1) of device columns `d` (an hbam_decode_split /
        hbam_split_next result): the fixed columns and each record's SAMRecordWritable bytes."""
        n = max(0, int(i1) - int(i0))
        out = {"n": n}
        for name, dt in FIXED:
            sz = np.dtype(dt).itemsize
            p = C.cast(getattr(d, name), C.c_void_p).value
            out[name] = self.download(p + int(i0) * sz, n * sz, dt).copy() if n else np.zeros(0, dt)
        ub = C.cast(d.ubuf, C.c_void_p).value
        out["records"] = [self.download(ub + int(o), 4 + int(b)).tobytes()
                          for o, b in zip(out["rec_off"], out["block_size"])]
        return out

    def decode_split_device(self, data, v_start, v_end, n_ref, comp_base=0, file_len=None):
        """Device-resident decode (bench path): returns the hbam_columns struct."""
        p, n, dev, keep = self._ptr(data)
        if file_len is None:
            file_len = comp_base + n
        d = Columns()
        rc = self.L.hbam_decode_split(self.h, p, dev, comp_base, n, file_len, v_start, v_end,
                                      n_ref, C.byref(d))
        return rc, d

    def guess_batch(self, data, beg, end, n_ref):
        p, n, dev, keep = self._ptr(data)
        beg = np.ascontiguousarray(beg, np.int64)
        end = np.ascontiguousarray(end, np.int64)
        k = len(beg)
        out = np.zeros(max(k, 1), np.int64)
        err = np.zeros(max(k, 1), np.int32)
        rc = self.L.hbam_guess_batch(self.h, p, dev, n, beg.ctypes.data, end.ctypes.data, k,
                                     n_ref, out.ctypes.data, err.ctypes.data)
        return rc, out[:k], err[:k]

    def guess_window_len(self, file_len, beg, end):
        return int(self.L.hbam_guess_window_len(int(file_len), int(beg), int(end)))

    def guess_bgzf_window_len(self, file_len, beg, end):
        return int(self.L.hbam_guess_bgzf_window_len(int(file_len), int(beg), int(end)))

    def guess_windows(self, windows, win_off, file_len, beg, end, n_ref):
        """hbam_guess_windows: windows = the k guess windows concatenated (win_off: k+1)."""
        p, n, dev, keep = self._ptr(windows)
        beg = np.ascontiguousarray(beg, np.int64)
        end = np.ascontiguousarray(end, np.int64)
        win_off = np.ascontiguousarray(win_off, np.uint64)
        k = len(beg)
        out = np.zeros(max(k, 1), np.int64)
        err = np.zeros(max(k, 1), np.int32)
        rc = self.L.hbam_guess_windows(self.h, p, dev, win_off.ctypes.data, int(file_len), beg.ctypes.data,
                                       end.ctypes.data, k, n_ref, out.ctypes.data, err.ctypes.data)
        return rc, out[:k], err[:k]

    def guess_bgzf_window(self, window, file_len, beg, end):
        p, n, dev, keep = self._ptr(window)
        e = C.c_int32(0)
        r = self.L.hbam_guess_bgzf_window(self.h, p, dev, n, int(file_len), int(beg), int(end), C.byref(e))
        return r, e.value

    def probabilistic_splits_windows(self, head, windows, win_off, file_len, beg, end):
        hp, hn, hdev, hkeep = self._ptr(head)
        if hdev:
            raise ValueError("the header prefix is a host buffer")
        p, n, dev, keep = self._ptr(windows)
        beg = np.ascontiguousarray(beg, np.uint64)
        end = np.ascontiguousarray(end, np.uint64)
        win_off = np.ascontiguousarray(win_off, np.uint64)
        k = len(beg)
        vs = np.zeros(max(k, 1), np.uint64)
        ve = np.zeros(max(k, 1), np.uint64)
        r = self.L.hbam_probabilistic_splits_windows(self.h, hp, hn, p, dev, win_off.ctypes.data, int(file_len),
                                                     beg.ctypes.data, end.ctypes.data, k, vs.ctypes.data,
                                                     ve.ctypes.data)
        if r < 0:
            return r, None, None
        return r, vs[:r], ve[:r]

    def guess_bgzf_block_start(self, data, beg, end):
        p, n, dev, keep = self._ptr(data)
        e = C.c_int32(0)
        r = self.L.hbam_guess_bgzf_block_start(self.h, p, dev, n, beg, end, C.byref(e))
        return r, e.value

    def probabilistic_splits(self, data, beg, end):
        p, n, dev, keep = self._ptr(data)
        beg = np.ascontiguousarray(beg, np.uint64)
        end = np.ascontiguousarray(end, np.uint64)
        k = len(beg)
        vs = np.zeros(max(k, 1), np.uint64)
        ve = np.zeros(max(k, 1), np.uint64)
        r = self.L.hbam_probabilistic_splits(self.h, p, dev, n, beg.ctypes.data, end.ctypes.data,
                                             k, vs.ctypes.data, ve.ctypes.data)
        if r < 0:
            return r, None, None
        return r, vs[:r], ve[:r]

    def splitting_index(self, data, granularity=4096):
        """SplittingBAMIndexer over a whole BAM file on the device -> uint64 entries."""
        p, n, dev, keep = self._ptr(data)
        h = self.parse_header(data)
        if not isinstance(h, dict):
            return h, None
        d = Columns()
        rc = self.L.hbam_decode_split(self.h, p, dev, 0, n, n, h["first_voffset"],
                                      (n << 16) | 0xffff, h["n_ref"], C.byref(d))
        if rc:
            return rc, None
        cap = int(d.n_records) // granularity + 2
        out = np.zeros(cap, np.uint64)
        r = self.L.hbam_splitting_index(self.h, C.byref(d), granularity, n, out.ctypes.data, cap)
        if r < 0:
            return int(r), None
        return 0, out[:r]

    def resolve_tokens(self, tokens, bitmap, tail_token=0, tail_dist=0):
        """Diagnostic: run the LZ77 pass on one token block -> (rc, status, resolved bytes)."""
        io = np.ascontiguousarray(np.frombuffer(bytes(tokens), np.uint8)).copy()
        bm = np.ascontiguousarray(bitmap, np.uint32)
        st = C.c_int32(0)
        rc = self.L.hbam_resolve_tokens(self.h, io.ctypes.data, len(io), bm.ctypes.data,
                                        tail_token, tail_dist, C.byref(st))
        return rc, st.value, io.tobytes()

    def bgzf_block_index(self, data, granularity=1):
        """BGZFBlockIndexer.index (util/BGZFBlockIndexer.java:97-181) on the device ->
        (rc, uint64 entries)."""
        p, n, dev, keep = self._ptr(data)
        cap = n // 28 // max(int(granularity), 1) + 2  # a BGZF block is at least 28 bytes
        out = np.zeros(cap, np.uint64)
        r = self.L.hbam_bgzf_block_index(self.h, p, dev, n, int(granularity), out.ctypes.data, cap)
        if r < 0:
            return int(r), None
        return 0, out[:r]

    # ---- read-name / CIGAR keyed consumers --------------------------------
    def _d2h(self, ptr, n, dtype):
        """Copy n elements of a device array (context-owned) to a numpy array."""
        out = np.empty(n, dtype)
        if n:
            rc = self.L.hbam_download(self.h, C.c_void_p(ptr), out.nbytes, C.c_void_p(out.ctypes.data))
            if rc:
                raise RuntimeError("hbam_download failed (%d): %s" % (rc, self.last_error()))
        return out

    def summarize_ranges(self, dcols):
        """SummarizeRecordReader's ranges over device columns (hbam_summarize_ranges) -> dict of
        numpy arrays + status."""
        r = RangesC()
        rc = self.L.hbam_summarize_ranges(self.h, C.byref(dcols), C.byref(r))
        if rc:
            raise RuntimeError("hbam_summarize_ranges failed (%d): %s" % (rc, self.last_error()))
        n = int(r.n)
        return dict(key=self._d2h(r.key, n, np.int64), beg=self._d2h(r.beg, n, np.int32),
                    end=self._d2h(r.end, n, np.int32), rev=self._d2h(r.rev, n, np.uint8),
                    record=self._d2h(r.record, n, np.uint32), status=int(r.status))

    def name_order(self, ubuf_ptr, rec_off_ptr, n, perm_ptr):
        rc = self.L.hbam_name_order(self.h, C.c_void_p(ubuf_ptr), C.c_void_p(rec_off_ptr), n,
                                    C.c_void_p(perm_ptr))
        if rc:
            raise RuntimeError("hbam_name_order failed (%d): %s" % (rc, self.last_error()))

    def fixmate(self, ubuf_ptr, rec_off_ptr, n):
        """FixMateReducer over the name shuffle of n device records -> host dict(payload,
        offsets, src, mate, n_groups, status)."""
        r = FixmateRunC()
        rc = self.L.hbam_fixmate(self.h, C.c_void_p(ubuf_ptr), C.c_void_p(rec_off_ptr), n, C.byref(r))
        if rc:
            raise RuntimeError("hbam_fixmate failed (%d): %s" % (rc, self.last_error()))
        k = int(r.n)
        return dict(payload=self._d2h(r.payload, int(r.payload_bytes), np.uint8),
                    offsets=self._d2h(r.offsets, k + 1, np.uint64) if k else np.zeros(1, np.uint64),
                    src=self._d2h(r.src, k, np.uint32), mate=self._d2h(r.mate, k, np.uint32),
                    n_groups=int(r.n_groups), status=int(r.status))

    # ---- BCF over BGZF --------------------------------------------------------
    def bcf_parse_header(self, file_prefix):
        """BCF2Codec.readHeader over the file's first bytes -> dict, or an error code."""
        a = np.ascontiguousarray(np.frombuffer(bytes(file_prefix), np.uint8))
        h = BcfHeaderC()
        rc = self.L.hbam_bcf_parse_header(self.h, C.c_void_p(a.ctypes.data), a.size, C.byref(h))
        if rc:
            return rc
        return dict(n_contig=h.n_contig, n_sample=h.n_sample, n_dict=h.n_dict, bgzf=bool(h.bgzf),
                    header_len=h.header_len, first_voffset=h.first_voffset)

    @staticmethod
    def _bcf_hdr(h):
        c = BcfHeaderC()
        c.n_contig, c.n_sample, c.n_dict = h["n_contig"], h["n_sample"], h["n_dict"]
        c.bgzf = int(bool(h["bgzf"]))
        c.header_len = int(h["header_len"])
        c.first_voffset = int(h.get("first_voffset", 0))
        return c

    def guess_bcf_window_len(self, file_len, beg, end, bgzf):
        return int(self.L.hbam_guess_bcf_window_len(int(file_len), int(beg), int(end), int(bool(bgzf))))

    def guess_bcf_windows(self, windows, win_off, file_len, beg, end, h):
        """hbam_guess_bcf_windows: BCFSplitGuesser over the k windows -> (rc, out, err)."""
        p, n, dev, keep = self._ptr(windows)
        beg = np.ascontiguousarray(beg, np.int64)
        end = np.ascontiguousarray(end, np.int64)
        win_off = np.ascontiguousarray(win_off, np.uint64)
        k = len(beg)
        out = np.zeros(max(k, 1), np.int64)
        err = np.zeros(max(k, 1), np.int32)
        hc = self._bcf_hdr(h)
        rc = self.L.hbam_guess_bcf_windows(self.h, p, dev, win_off.ctypes.data, int(file_len), beg.ctypes.data,
                                           end.ctypes.data, k, C.byref(hc), out.ctypes.data, err.ctypes.data)
        return rc, out[:k], err[:k]

    def bcf_decode_split(self, data, h, start, end_or_len, comp_base=0, file_len=None, keep_data=False):
        """BCFRecordReader over one split (hbam_bcf_decode_split) -> host numpy columns."""
        p, n, dev, keep = self._ptr(data)
        if file_len is None:
            file_len = comp_base + n
        d = BcfColumnsC()
        hc = self._bcf_hdr(h)
        rc = self.L.hbam_bcf_decode_split(self.h, p, dev, int(comp_base), n, int(file_len), C.byref(hc),
                                          int(start), int(end_or_len), C.byref(d))
        if rc:
            return {"rc": rc, "error": self.last_error()}
        k = int(d.n_records)
        out = {"rc": 0, "n": k, "status": int(d.status), "err_record": int(d.err_record)}
        for name, dt in BCF_FIELDS:
            out[name] = self._d2h(getattr(d, name), k, dt)
        if keep_data:
            out["data"] = self._d2h(d.data, int(d.data_len), np.uint8)
        out["timing"] = self.timing()
        return out
