"""Multi-GPU sharded decode of one BAM file.

One process per GPU (torch.distributed; RCCL on the GPU box, gloo in CPU tests).  The file's
Hadoop FileSplits are dealt to ranks as contiguous byte ranges; every rank guesses the record
starts of ITS FileSplits (BAMSplitGuesser, one device launch), the guesses are all-gathered
(one int64 per split — the only exchange), and every rank then applies
BAMInputFormat.addProbabilisticSplits' merge rule (BAMInputFormat.java:181-222: a split whose
guess returns `end` extends its predecessor's vEnd, possibly across a rank boundary) to the
global list, so the FileVirtualSplits are exactly the reference's.  Each rank then decodes the
virtual splits derived from its FileSplits; nothing else crosses ranks.
"""
import numpy as np


def file_splits(file_len, split_size):
    """Hadoop 1.2.1 FileInputFormat split sizing (SPLIT_SLOP 1.1) -> (beg, end) arrays."""
    beg, end, rem = [], [], file_len
    while split_size > 0 and rem / split_size > 1.1:
        beg.append(file_len - rem)
        end.append(file_len - rem + split_size)
        rem -= split_size
    if rem:
        beg.append(file_len - rem)
        end.append(file_len)
    return np.array(beg, np.int64), np.array(end, np.int64)


def owner_ranges(n_splits, world):
    """Contiguous split index ranges [lo, hi) per rank (balanced)."""
    q, r = divmod(n_splits, world)
    out, lo = [], 0
    for k in range(world):
        hi = lo + q + (1 if k < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


def merge_guesses(beg, end, guess):
    """addProbabilisticSplits merge rule over the global guess list.
    Returns (v_start, v_end, owner_split_index) arrays, or raises IOError for an empty
    first split (the reference's "no reads in first split")."""
    vs, ve, own = [], [], []
    for i in range(len(beg)):
        aligned_end = (int(end[i]) << 16) | 0xffff
        if int(guess[i]) == int(end[i]):
            if not vs:
                raise IOError("no reads in first split: bad BAM file or tiny split size?")
            ve[-1] = aligned_end
        else:
            vs.append(int(guess[i]))
            ve.append(aligned_end)
            own.append(i)
    return np.array(vs, np.uint64), np.array(ve, np.uint64), np.array(own, np.int64)


def sharded_virtual_splits(file_len, split_size, rank, world, guess_fn, all_gather_fn):
    """Global FileVirtualSplits, computed cooperatively.
    guess_fn(beg_array, end_array) -> guesses for this rank's FileSplits;
    all_gather_fn(local_int64_array) -> concatenation over ranks (in rank order)."""
    beg, end = file_splits(file_len, split_size)
    lo, hi = owner_ranges(len(beg), world)[rank]
    local = np.asarray(guess_fn(beg[lo:hi], end[lo:hi]), np.int64) if hi > lo else np.zeros(0, np.int64)
    guesses = all_gather_fn(local)
    assert len(guesses) == len(beg)
    vs, ve, own = merge_guesses(beg, end, guesses)
    mine = (own >= lo) & (own < hi)
    return vs[mine], ve[mine], (vs, ve)


def torch_all_gather_fn(dist, device):
    """all_gather of variable-length int64 arrays through torch.distributed."""
    import torch

    def f(local):
        world = dist.get_world_size()
        n = torch.tensor([len(local)], dtype=torch.int64, device=device)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n)
        mx = int(max(int(s.item()) for s in sizes))
        buf = torch.zeros(max(mx, 1), dtype=torch.int64, device=device)
        if len(local):
            buf[:len(local)] = torch.from_numpy(np.asarray(local, np.int64)).to(device)
        outs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf)
        return np.concatenate([o[:int(s.item())].cpu().numpy() for o, s in zip(outs, sizes)])
    return f
