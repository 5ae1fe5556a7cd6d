"""Sharded single merge: one composition spread over the GPUs of a node.

The reference composes two branch logs in one sequential loop (semmerge/compose.py:11-114).
Its output order T is (precedence, timestamp, id, side, index): kind-major, so a shard that
owns every op of both branches whose key falls in a key range owns, for each kind, one
contiguous piece of T, and the pieces of the shards follow each other in shard order.  One
process per GPU; the steps of one merge and the collectives each one uses:

1. exchange   each rank starts with an index slice of each branch log (how the logs are
              loaded).  Timestamp-ordered logs (lift.ts emits them) are split by timestamp
              range: one all_gather of 8 words per rank, splitters and per-destination
              counts on the device, one all_gather of the counts (the one host sync: the
              all-to-all needs its split sizes), then ONE all_to_all_single of packed 37-B
              op records; only the ops near the slice edges move.  Logs in any order take
              a sample sort instead: an all_gather of key samples, splitters on the full
              T key, one all_gather of counts, one all_to_all_single of 41-B records
              (with the op's global index).
2. order      smx_shard_step(ORDER): the single-GPU plan + window kernels on the shard
              (asynchronous on the presorted plan), then one all_gather of the summary
              and the halo exports; the halo is assembled on the device.
3. walk       the DivergentRename walk (compose.py:60-70, 88-98) with the halo (the next
              renames of each branch on the following shards) and the incoming open
              region held on the device; one all_gather of the summaries and one host
              read per round; a shard whose incoming region changed re-runs (rare).
4. tables     per-symbol last writers (compose.py:27-28, 71-82, 99-110): partial tables
              tagged (shard + 1) << 32, with the value widths appended, in ONE MAX
              all_reduce.  Moves with a None value add an all_gather of the move tables
              (the lower shards' prefix).
5. emit       composed output per shard; order[] and conflicts hold global source indices.

Collectives run on device tensors over RCCL ("nccl"); on "gloo" (the CPU tests and
multi-rank tests on one GPU) they go through host copies.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from ._lib import _ptr, check, lib

FIELDS = ("kind", "ts", "hi", "lo", "sym", "v0", "v1")
S_KINDS, S_REN, S_MVNONE, S_FAIL = 0, 18, 20, 21
S_OPEN, S_AHEAD, S_D, S_NCONF, S_NSKIP, S_OVER, S_WIDTH = 22, 23, 24, 25, 26, 27, 28
S_TABOVER = 31   # a value too wide for the 32-bit partial tables (smx_shard.tab32)
TAB32_MAX_BITS = 8  # the widest rank tag smx_shard_step accepts in 32-bit entries (smx_compose.hip TABLES)


def tab32_bits(world: int) -> int:
    """Tag bits of the 32-bit partial tables for `world` ranks (the tag is rank + 1), or 0
    when the tag does not fit the library's limit: those worlds keep the 64-bit tables."""
    b = int(world).bit_length()
    return b if b <= TAB32_MAX_BITS else 0
N_KINDS = 18
SUM = _abi.SHARD_SUMMARY
I64_MIN = -(2 ** 63)
RH = 32  # keys from each end of each branch slice in the range info (host-side cuts)

# packed exchange record: ts, hi, lo (8 B each), sym, v0, v1 (4 B), kind (1 B) = 37 B;
# the sample-sort exchange appends the op's global source index (4 B) = 41 B
REC_FIELDS = ("ts", "hi", "lo", "sym", "v0", "v1", "kind")


class Comm:
    """Collectives on device tensors: direct on RCCL, through host copies otherwise."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.direct = dist.get_backend(group) == "nccl"

    def _host(self, t):
        return t if self.direct else t.cpu()

    def all_gather(self, t):
        """[world, *t.shape] tensor on t's device."""
        import torch
        x = self._host(t.contiguous())
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, x, group=self.group) if self.direct else \
            self.dist.all_gather(list(out.unbind(0)), x, group=self.group)
        return out.to(t.device)

    def all_reduce_max(self, t) -> None:
        x = self._host(t)
        self.dist.all_reduce(x, op=self.dist.ReduceOp.MAX, group=self.group)
        if x is not t:
            t.copy_(x)

    def all_to_all(self, t, in_splits: Sequence[int], out_splits: Sequence[int]):
        """Rows of t (dim 0) to the ranks: in_splits rows to each, out_splits from each."""
        import torch
        x = self._host(t.contiguous())
        out = torch.empty((int(sum(out_splits)),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self.dist.all_to_all_single(out, x, list(map(int, out_splits)), list(map(int, in_splits)),
                                    group=self.group)
        return out.to(t.device)


@dataclass
class BranchSlice:
    """This rank's index slice [start, start + n) of one branch log (device tensors)."""
    start: int
    kind: object
    ts: object
    hi: object
    lo: object
    sym: object
    v0: object
    v1: object

    @property
    def n(self) -> int:
        return int(self.kind.numel())


def slices_from_soa(soa, rank: int, world: int, device) -> Tuple[BranchSlice, BranchSlice, int, int]:
    """Rank's even index slices of both branches of a global SoA (tests, small merges)."""
    import torch

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(device)

    out = []
    for side, (lo_i, n_s) in enumerate(((0, soa.n_a), (soa.n_a, soa.n_b))):
        s0, s1 = n_s * rank // world, n_s * (rank + 1) // world
        sl = slice(lo_i + s0, lo_i + s1)
        out.append(BranchSlice(s0, up(soa.kind[sl], np.uint8), up(soa.ts[sl], np.int64),
                               up(soa.oid_hi[sl], np.int64), up(soa.oid_lo[sl], np.int64),
                               up(soa.sym[sl], np.int32), up(soa.v0[sl], np.int32),
                               up(soa.v1[sl], np.int32)))
    return out[0], out[1], soa.n_a, soa.n_b


def _u64_key(t):
    """int64 tensor holding u64 payloads -> order-preserving signed image."""
    return t ^ I64_MIN


def pack_records(cols: dict, gidx=None):
    """Field tensors of m ops -> uint8 [m, 37] (or [m, 41] with gidx) packed records."""
    import torch
    m = int(cols["kind"].numel())
    parts = [cols[f].contiguous().view(torch.uint8).reshape(m, cols[f].element_size()) for f in REC_FIELDS]
    if gidx is not None:
        parts.append(gidx.contiguous().view(torch.uint8).reshape(m, 4))
    return torch.cat(parts, dim=1)


def unpack_records(rec, dtypes: dict, with_gidx: bool = False):
    """uint8 [m, R] records -> (dict of field tensors, gidx int32 or None)."""
    import torch
    m = int(rec.shape[0])

    def col(o, w, dt):  # a fresh aligned copy of the byte columns [o, o + w)
        t = torch.empty((m, w), dtype=torch.uint8, device=rec.device)
        t.copy_(rec[:, o:o + w])
        return t.view(dt).reshape(-1)

    out, o = {}, 0
    for f in REC_FIELDS:
        w = torch.empty(0, dtype=dtypes[f]).element_size()
        out[f] = col(o, w, dtypes[f])
        o += w
    g = col(o, 4, torch.int32) if with_gidx else None
    return out, g


def lex_dest(keys: Sequence, splitters):
    """Shard of each op: the number of splitters (rows of `splitters`, [k, len(keys)])
    at or below the op's key tuple, compared lexicographically."""
    import torch
    n = int(keys[0].numel())
    k = int(splitters.shape[0])
    gt = torch.zeros((n, k), dtype=torch.bool, device=keys[0].device)
    eq = torch.ones((n, k), dtype=torch.bool, device=keys[0].device)
    for i, key in enumerate(keys):
        col = key.view(n, 1)
        s = splitters[:, i].view(1, k)
        gt |= eq & (col > s)
        eq &= col == s
    return (gt | eq).sum(dim=1)


class ShardedCompose:
    """One rank's part of a sharded merge.  `a`, `b`: this rank's index slices of the
    global branch logs, na_glob / nb_glob the global branch sizes.

    mode "range" (timestamp-ordered logs): the slices are copied once into field buffers
    with `headroom` free entries on both sides of each branch range; the exchange writes
    the ops arriving from the neighbouring shards into the headroom, so the ops that stay
    (nearly all of them) never move, and the shard is handed to the kernels in place: A'
    at [a_lo, a_hi) and B' at [b_lo, b_hi) of every field buffer, B' after a gap
    (smx_ops.b_gap).  mode "sample" (logs in any order): a sample-sort exchange into
    contiguous shard buffers, with a global source map (smx_shard.src_map) and the
    generic sorting plan.  "auto" picks range when every slice is ordered."""

    def __init__(self, a: BranchSlice, b: BranchSlice, na_glob: int, nb_glob: int, n_sym: int,
                 comm: Comm, device, halo_cap: int = 4096, headroom: Optional[int] = None,
                 restore: bool = True, mode: str = "auto", oversample: int = 64) -> None:
        import torch
        if mode not in ("auto", "range", "sample"):
            raise ValueError(f"mode {mode!r}")
        self.torch = torch
        self.mode = mode
        self.oversample = oversample
        self.na_glob, self.nb_glob = na_glob, nb_glob
        self.n_sym = n_sym
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self.dev = torch.device(device)
        self.H = halo_cap
        self.restore = restore
        self.na_s, self.nb_s = a.n, b.n
        self.a_start, self.b_start = a.start, b.start
        self.dtypes = {f: getattr(a, f).dtype for f in FIELDS}
        hd = headroom if headroom is not None else max(1 << 16, (a.n + b.n) // 32)
        self._alloc(hd, a, b)
        self._ws = None
        self._ws_bytes = 0
        self._outn = -1
        self._saved = []
        self.sbuf, self.src_map = None, None
        dv = self.dev
        H2 = 2 * max(self.H, 1)
        # the summary and the halo exports (sym, cls, src) in one buffer: the order
        # exchange gathers it as it is
        self._sx = torch.zeros(SUM + 3 * H2 // 2, dtype=torch.int64, device=dv)
        self.summary = self._sx[:SUM]
        self.xport = self._sx[SUM:].view(torch.int32).view(3, H2)
        self.halo = torch.zeros((2, 3, max(self.H, 1)), dtype=torch.int32, device=dv)
        self.halo_dev = torch.zeros(4, dtype=torch.int64, device=dv)
        self.in_state = (0, 0)
        self.in_dev = torch.zeros(2, dtype=torch.int64, device=dv)
        # partial tables [3][n_sym] then the 3 value widths: one MAX all_reduce for both
        self.part = torch.zeros(3 * max(n_sym, 1) + 3, dtype=torch.int64, device=dv)
        self.glob = self.part[3 * max(n_sym, 1):]
        # the same tables with 32-bit entries: the rank tag in the top bits under a clear
        # sign bit (an int32 MAX keeps the last writer) -- half the all-reduce's bytes
        # whenever every value fits the rest (include/smx.h smx_shard.tab32)
        self.tab_bits = tab32_bits(self.world)
        self.part32 = torch.zeros(3 * max(n_sym, 1) + 3, dtype=torch.int32, device=dv) \
            if self.tab_bits else None
        self.tab32_used = 0  # tables steps that ran with 32-bit entries (tests, probes)
        self.emit_redo = 0   # steps whose speculative tables and EMIT were redone
        self.tab_redo = 0    # steps whose 32-bit tables overflowed and were redone with 64-bit entries
        self.n_xchg = 0      # ops this rank received from other ranks in the last exchange
        self.order_fixes = 0  # ORDER_FIX runs (dense timestamp ties) on this rank
        # every timestamp below 2^63 (ISO keys, dense ranks): the signed int64 order of
        # the stored words is the u64 order, so the splitter search needs no key copy
        self._ts_signed = [bool((self._orig(br, "ts") >= 0).all()) for br in range(2)]
        self._sizes = torch.tensor([self.na_s, self.nb_s], dtype=torch.int64, device=dv)
        self._one = torch.ones(1, dtype=torch.int64, device=dv)
        self._zero2 = torch.zeros(2, dtype=torch.int64, device=dv)
        self._signed = torch.tensor([int(x) for x in self._ts_signed], dtype=torch.int64, device=dv)
        self._bind_key = None
        self._halo_key = None
        self._info_key = None
        self._info_out = None  # smx_shard_range_info's output (int64 [9 + 4 RH])
        self.host_cut_plans = 0  # exchanges planned from the gathered head / tail keys alone

    def _alloc(self, hd: int, a, b) -> None:
        """Field buffers [hd | A slice | 2 hd | B slice | hd]; a, b: BranchSlices or the
        previous buffers (grow)."""
        torch = self.torch
        self.hd = hd
        self.capA = self.na_s + 2 * hd
        cap = self.capA + self.nb_s + 2 * hd
        old = getattr(self, "buf", None)
        self.buf = {}
        for f in FIELDS:
            src_a = getattr(a, f) if old is None else old[f][self._oa: self._oa + self.na_s]
            src_b = getattr(b, f) if old is None else old[f][self._ob: self._ob + self.nb_s]
            t = torch.zeros(cap, dtype=src_a.dtype, device=self.dev)
            t[hd: hd + self.na_s] = src_a
            t[self.capA + hd: self.capA + hd + self.nb_s] = src_b
            self.buf[f] = t
        self._oa, self._ob = hd, self.capA + hd   # original slices in the buffers

    # -- 1. exchange ------------------------------------------------------------------
    def _orig(self, br: int, f: str):
        return self.buf[f][self._oa: self._oa + self.na_s] if br == 0 else \
            self.buf[f][self._ob: self._ob + self.nb_s]

    def _info_index(self):
        """Buffer positions of the range info's keys: the first and last key of each
        branch slice, then RH keys from the head and RH from the tail of each (the tail
        right-aligned; short slices repeat their first position as padding)."""
        ends, edges, live_e, live_g = [], [], [], []
        for o, n in ((self._oa, self.na_s), (self._ob, self.nb_s)):
            ends += [o, o + n - 1] if n else [0, 0]
            live_e += [n > 0] * 2
            h = min(RH, n)
            pad = [o if n else 0]
            edges += [o + i for i in range(h)] + pad * (RH - h)
            edges += pad * (RH - h) + [o + n - h + i for i in range(h)]
            live_g += [n > 0] * (2 * RH)
        # an empty slice's entries read key 0, as k_range_info writes them
        self._info_live = self.torch.tensor(live_e + live_g, dtype=self.torch.bool, device=self.dev)
        return self.torch.tensor(ends + edges, dtype=self.torch.int64, device=self.dev)

    def _range_info(self):
        """Device int64 [9 + 4 RH]: this rank's slice sizes, first / last key of each
        slice (u64 order as int64), whether the slices are ordered, per branch whether
        every timestamp is below 2^63 (the device cut search runs on the stored words),
        then the RH head and RH tail keys of each slice (host-side cuts)."""
        torch = self.torch
        check_order = self.mode == "auto"  # "range": the ORDER plan checks the order itself
        if self.dev.type == "cuda":  # two launches (smx_shard_range_info)
            if self._info_out is None:
                self._info_out = torch.empty(9 + 4 * RH, dtype=torch.int64, device=self.dev)
            s = torch.cuda.current_stream(self.dev).cuda_stream
            check(lib().smx_shard_range_info(self.buf["ts"].data_ptr(), self._oa, self.na_s, self._ob, self.nb_s,
                                             RH, int(check_order), int(self._ts_signed[0]),
                                             int(self._ts_signed[1]), self._info_out.data_ptr(), s))
            return self._info_out
        # the exchange protocol's CPU tests (gloo, host tensors): the same vector in torch
        if self._info_key != (self._oa, self._ob):
            self._info_idx = self._info_index()
            self._info_key = (self._oa, self._ob)
        keys = _u64_key(self.buf["ts"].index_select(0, self._info_idx)) * self._info_live
        ok = self._one
        if check_order:
            for br, n in ((0, self.na_s), (1, self.nb_s)):
                if n > 1:
                    k = _u64_key(self._orig(br, "ts"))
                    ok = ok & (k[1:] >= k[:-1]).all().to(torch.int64).view(1)  # both branches
        return torch.cat([self._sizes, keys[:4], ok, self._signed, keys[4:]])

    @staticmethod
    def _host_cuts(g: np.ndarray, tau: np.ndarray):
        """allc [W, 2, W] from the gathered range info alone, or None when a splitter
        falls between a slice's RH head and RH tail keys (then the device searches).
        Every (rank, branch, splitter) at once (a loop over the W x 2 slices cost ~0.5 ms
        of numpy calls per exchange at W = 8): a cut is the count of head keys below the
        splitter, or the slice length less RH plus the count of tail keys below it when
        the splitter lies past the head (keys sorted, so counts are searchsorted 'left')."""
        W = g.shape[0]
        n = g[:, 0:2]                                          # [W, 2] slice lengths
        keys = g[:, 9: 9 + 4 * RH].reshape(W, 2, 2, RH)       # [rank, branch, head / tail, RH]
        head, tail = keys[:, :, 0, :], keys[:, :, 1, :]
        t = tau[None, None, None, :]
        valid = np.arange(RH)[None, None, :] < np.minimum(n, RH)[:, :, None]  # (short slices: padding)
        ch = ((head[..., None] < t) & valid[..., None]).sum(axis=2)           # [W, 2, W-1]
        ct = (tail[..., None] < t).sum(axis=2)
        big = (n > RH)[:, :, None]
        in_head = tau[None, None, :] <= head[:, :, RH - 1:RH]  # every key below tau is in the head
        in_tail = tau[None, None, :] > tail[:, :, 0:1]         # every key before the tail is below tau
        if np.any(big & ~(in_head | in_tail)):
            return None
        nn = n[:, :, None]
        cuts = np.clip(np.where(big & ~in_head, nn - RH + ct, ch), 0, nn)
        return np.diff(np.concatenate([np.zeros_like(nn), cuts, nn], axis=2), axis=2)

    @staticmethod
    def _range_plan(g: np.ndarray):
        """Host, from every rank's _range_info (g [W, 9]): (ordered, tau) -- the key
        ranges' lower bounds tau[1..W-1] (shard r owns keys [tau_r, tau_r+1)), the
        running maximum of the ranks' first keys."""
        W = g.shape[0]
        ordered = bool(g[:, 6].min() == 1)
        for br in range(2):                 # slices of a branch must follow each other
            nz = g[:, br] > 0
            last = np.where(nz, g[:, 3 + 2 * br], I64_MIN)
            prev = np.concatenate([[I64_MIN], np.maximum.accumulate(last)[:-1]])
            ordered &= bool((~nz | (g[:, 2 + 2 * br] >= prev)).all())
        cand = np.where(g[:, 0] > 0, g[:, 2], np.where(g[:, 1] > 0, g[:, 4], I64_MIN)).astype(np.int64)
        cand[0] = I64_MIN
        return ordered, np.maximum.accumulate(cand)[1:] if W > 1 else np.zeros(0, np.int64)

    def _range_counts(self):
        """allc [W, 2, W] (src, branch, dest) op counts of the key-range split, or None when
        the logs are not timestamp-ordered.  One host sync: the gathered range info
        carries RH keys from each end of every slice, and a splitter (the running maximum
        of the ranks' first keys) cuts a timestamp-ordered slice near one of its ends
        unless the slices are badly skewed, so every rank computes every cut on the host.
        Otherwise a second sync: every rank's cut positions from binary searches on the
        device.  (Planning on the device, to save the sync, measured slower: a dozen tiny
        torch launches cost more than the sync, profiles/r03_c/shard_probe.txt.)"""
        torch = self.torch
        W = self.world
        g = self.comm.all_gather(self._range_info()).cpu().numpy()        # [W, 9 + 4 RH]
        ordered, tau = self._range_plan(g)
        if not ordered:
            return None
        allc = self._host_cuts(g, tau)
        if allc is not None:  # the common case: one host sync for the whole plan
            self.host_cut_plans += 1
            return allc
        cuts = torch.zeros((2, max(W - 1, 1)), dtype=torch.int64, device=self.dev)
        if W > 1:
            tk = torch.from_numpy(tau).to(self.dev)
            for br, n in ((0, self.na_s), (1, self.nb_s)):
                if n:
                    ts = self._orig(br, "ts")
                    # every timestamp below 2^63: search the stored words (int64 order =
                    # u64 order); a splitter above 2^63 (key >= 0) is fixed on the host
                    cuts[br] = torch.searchsorted(ts, _u64_key(tk)) if self._ts_signed[br] else \
                        torch.searchsorted(_u64_key(ts).contiguous(), tk)
        gc = self.comm.all_gather(cuts).cpu().numpy()                      # [W, 2, W-1]
        allc = np.zeros((W, 2, W), np.int64)
        for q in range(W):
            for br in range(2):
                n = int(g[q, br])
                c = gc[q, br, : W - 1].copy()
                if W > 1 and g[q, 7 + br]:  # a splitter above every stored word
                    c[tau >= 0] = n
                edges = np.concatenate([[0], np.clip(c, 0, n), [n]]) if W > 1 else np.array([0, n])
                allc[q, br] = np.diff(edges)
        return allc

    def exchange(self) -> None:
        """Every op to the shard owning its key (collective)."""
        self._saved = []
        if self.mode != "sample":
            allc = self._range_counts()
            if allc is not None:
                self.exchange_mode = "range"
                self._exchange_range(allc)
                return
            if self.mode == "range":
                raise ValueError("sharded merge (mode 'range') needs timestamp-ordered branch logs "
                                 "(a slice is unordered or a branch decreases across rank slices)")
        self.exchange_mode = "sample"
        self._exchange_sample()

    def _exchange_range(self, allc: np.ndarray) -> None:
        """allc[src, branch, dest]: op counts of the key-range split."""
        torch = self.torch
        r, W = self.rank, self.world
        send, recv = allc[r], allc[:, :, r]                              # [br, dest], [src, br]
        lo_s, hi_s = send[:, :r].sum(axis=1), send[:, r + 1:].sum(axis=1)
        lo_r, hi_r = recv[:r].sum(axis=0), recv[r + 1:].sum(axis=0)
        need = int(max(0, (lo_r - lo_s).max(), (hi_r - hi_s).max()))
        if need > self.hd:  # skewed slices: grow the headroom (copies the slices once)
            self._alloc(need + (self.na_s + self.nb_s) // 32, None, None)
        first = [int(allc[:, br, :r].sum()) for br in range(2)]
        self.src_a = first[0]
        self.src_b = self.na_glob + first[1]
        n0 = (self.na_s, self.nb_s)
        base = (self._oa, self._ob)
        self.rng = [(base[br] + int(lo_s[br] - lo_r[br]), base[br] + n0[br] - int(hi_s[br] - hi_r[br]))
                    for br in range(2)]
        in_splits = [0 if d == r else int(send[0, d] + send[1, d]) for d in range(W)]
        out_splits = [0 if q == r else int(recv[q, 0] + recv[q, 1]) for q in range(W)]
        self.n_xchg = int(sum(out_splits))
        moving = int(allc.sum()) - sum(int(allc[q, :, q].sum()) for q in range(W))
        if moving:  # the same decision on every rank: the all-to-all is collective
            soff = [np.concatenate([[0], np.cumsum(send[br])]) for br in range(2)]
            cols = {}
            for f in REC_FIELDS:
                pieces = [self._orig(br, f)[soff[br][d]: soff[br][d + 1]]
                          for d in range(W) if d != r for br in range(2)]
                cols[f] = torch.cat(pieces) if pieces else self.buf[f][:0]
            got = self.comm.all_to_all(pack_records(cols), in_splits, out_splits)
            f_in, _ = unpack_records(got, self.dtypes)
            roff = np.concatenate([[0], np.cumsum(out_splits)])
            # every arriving op's (received row, buffer position): the lower ranks' ops of a
            # branch go below its slice, the higher ranks' above; one index copy to the
            # device and one gather / scatter per field (not one per branch and side)
            src, dst = [], []
            for br in range(2):
                for qs, dst0 in ((range(r), self.rng[br][0]),
                                 (range(r + 1, W), base[br] + n0[br] - int(hi_s[br]))):
                    ii = [np.arange(roff[q] + (recv[q, 0] if br else 0),
                                    roff[q] + (recv[q, 0] if br else 0) + recv[q, br]) for q in qs]
                    ii = np.concatenate(ii) if ii else np.zeros(0, np.int64)
                    src.append(ii)
                    dst.append(np.arange(dst0, dst0 + len(ii)))
            sd = np.stack([np.concatenate(src), np.concatenate(dst)]).astype(np.int64)
            if sd.shape[1]:
                sd = torch.from_numpy(sd).to(self.dev)
                ix, at = sd[0], sd[1]
                for f in FIELDS:
                    if self.restore:  # originals under the arriving ops, put back after the step
                        self._saved.append((f, at, self.buf[f][at]))
                    self.buf[f][at] = f_in[f][ix]
        self.n_a = self.rng[0][1] - self.rng[0][0]
        self.n_b = self.rng[1][1] - self.rng[1][0]
        self._fields = self.buf
        self._map_on = False
        self._bind()

    def _keys(self):
        """Full T keys of this rank's ops, A slice then B slice: kind (precedence rank),
        ts, oid hi, oid lo (u64 as ordered int64) and the global source index (side,
        then index within the branch)."""
        torch = self.torch
        cat = torch.cat
        kind = cat([self._orig(0, "kind"), self._orig(1, "kind")]).to(torch.int64)
        ts = _u64_key(cat([self._orig(0, "ts"), self._orig(1, "ts")]))
        hi = _u64_key(cat([self._orig(0, "hi"), self._orig(1, "hi")]))
        lo = _u64_key(cat([self._orig(0, "lo"), self._orig(1, "lo")]))
        gidx = cat([torch.arange(self.a_start, self.a_start + self.na_s, device=self.dev),
                    torch.arange(self.na_glob + self.b_start, self.na_glob + self.b_start + self.nb_s,
                                 device=self.dev)])
        return [kind, ts, hi, lo, gidx]

    def _exchange_sample(self) -> None:
        """Sample sort on the full T key: all_gather of samples, splitters (device), one
        all_gather of the counts (host sync), one all_to_all of 41-B records."""
        torch = self.torch
        r, W, dv = self.rank, self.world, self.dev
        keys = self._keys()
        n = self.na_s + self.nb_s
        S = self.oversample * W
        samp = torch.ones((S, 6), dtype=torch.int64, device=dv)         # col 0: 0 = valid
        k = min(n, S)
        if k:
            pos = torch.arange(k, device=dv) * n // k                    # evenly spaced
            samp[:k, 0] = 0
            for i, key in enumerate(keys):
                samp[:k, 1 + i] = key[pos]
        allS = self.comm.all_gather(samp).reshape(W * S, 6)
        order = torch.arange(W * S, device=dv)
        for c in range(5, -1, -1):                                        # lexsort, last key first
            order = order[torch.sort(allS[order, c], stable=True).indices]
        srt = allS[order]
        nvalid = (allS[:, 0] == 0).sum()
        at = (torch.arange(1, W, device=dv) * nvalid // W).clamp(max=W * S - 1)
        split = srt[at, 1:]                                               # [W-1, 5]
        if n:
            dest = lex_dest(keys, split) if W > 1 else torch.zeros(n, dtype=torch.int64, device=dv)
            side = torch.cat([torch.zeros(self.na_s, dtype=torch.int64, device=dv),
                              torch.ones(self.nb_s, dtype=torch.int64, device=dv)])
            key2 = dest * 2 + side
            perm = torch.sort(key2, stable=True).indices
            cnt = torch.bincount(key2, minlength=2 * W)
        else:
            perm = torch.zeros(0, dtype=torch.int64, device=dv)
            cnt = torch.zeros(2 * W, dtype=torch.int64, device=dv)
        allc = self.comm.all_gather(cnt).cpu().numpy().reshape(W, W, 2)   # [src, dest, side]: host sync
        cols = {f: torch.cat([self._orig(0, f), self._orig(1, f)])[perm] for f in REC_FIELDS}
        rec = pack_records(cols, keys[4].to(torch.int32)[perm])
        in_splits = [int(allc[r, d].sum()) for d in range(W)]
        out_splits = [int(allc[q, r].sum()) for q in range(W)]
        self.n_xchg = int(sum(out_splits)) - int(allc[r, r].sum())
        got = self.comm.all_to_all(rec, in_splits, out_splits)
        f_in, g_in = unpack_records(got, self.dtypes, with_gidx=True)
        roff = np.concatenate([[0], np.cumsum(out_splits)])
        # A' then B': each source's A records then its B records, sources in rank order
        # (= global index order within each branch)
        ia = [np.arange(roff[q], roff[q] + allc[q, r, 0]) for q in range(W)]
        ib = [np.arange(roff[q] + allc[q, r, 0], roff[q + 1]) for q in range(W)]
        ii = np.concatenate(ia + ib).astype(np.int64)
        ix = torch.from_numpy(ii).to(dv)
        self.n_a = int(allc[:, r, 0].sum())
        self.n_b = int(allc[:, r, 1].sum())
        n_loc = self.n_a + self.n_b
        self._sbuf(n_loc)
        for f in FIELDS:
            self.sbuf[f][:n_loc] = f_in[f][ix]
        self.src_map[:n_loc] = g_in[ix]
        self.rng = [(0, self.n_a), (self.n_a, n_loc)]
        self.src_a, self.src_b = 0, self.na_glob
        self._fields = self.sbuf
        self._map_on = True
        self._bind()

    def _sbuf(self, n_loc: int) -> None:
        torch = self.torch
        if self.sbuf is None or self.sbuf["kind"].numel() < max(n_loc, 1):
            cap = max(n_loc + n_loc // 16, 1)
            self.sbuf = {f: torch.zeros(cap, dtype=self.dtypes[f], device=self.dev) for f in FIELDS}
            self.src_map = torch.zeros(cap, dtype=torch.int32, device=self.dev)

    def _compact(self) -> None:
        """A range shard as one contiguous [A' | B'] (b_gap = 0), so that ORDER_FIX may
        take the generic plan; sources stay src_a + j / src_b + j."""
        if self._fields is self.sbuf:
            return
        n_loc = self.n_a + self.n_b
        self._sbuf(n_loc)
        (a_lo, a_hi), (b_lo, b_hi) = self.rng
        for f in FIELDS:
            self.sbuf[f][:self.n_a] = self.buf[f][a_lo:a_hi]
            self.sbuf[f][self.n_a:n_loc] = self.buf[f][b_lo:b_hi]
        self.rng = [(0, self.n_a), (self.n_a, n_loc)]
        self._fields = self.sbuf
        self._map_on = False
        self._bind()

    def _restore(self) -> None:
        for f, at, t in reversed(self._saved):  # (at: buffer positions, t: their originals)
            self.buf[f][at] = t
        self._saved = []

    # -- device structs -----------------------------------------------------------------
    def _bind(self) -> None:
        torch = self.torch
        key = (self.n_a, self.n_b, tuple(map(tuple, self.rng)), self._fields["kind"].data_ptr(),
               self._map_on, self.src_a, self.src_b)
        if key == self._bind_key:  # the same layout as the last step (a repeated merge)
            return
        self._bind_key = key
        n = self.n_a + self.n_b
        if n > self._outn:
            nn = max(n, 1)
            self.order = torch.empty(nn, dtype=torch.int32, device=self.dev)
            self.addr = torch.empty(nn, dtype=torch.int32, device=self.dev)
            self.file = torch.empty(nn, dtype=torch.int32, device=self.dev)
            self.ctx = torch.empty(nn, dtype=torch.int32, device=self.dev)
            self._outn = n
        self.cap = max(min(self.n_a, self.n_b) + 2 * self.H, 1)
        if getattr(self, "conf", None) is None or self.conf.numel() < 2 * self.cap:
            self.conf = torch.empty(2 * self.cap, dtype=torch.int32, device=self.dev)
        self.counts = torch.zeros(2, dtype=torch.int64, device=self.dev)
        ws = C.c_size_t(0)
        check(lib().smx_compose_workspace_bytes(self.n_a, self.n_b, self.n_sym, C.byref(ws)))
        if ws.value > self._ws_bytes:
            self._ws = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=self.dev)
            self._ws_bytes = ws.value
        a_lo = self.rng[0][0]
        gap = self.rng[1][0] - self.rng[0][1]
        fb = self._fields
        fp = {f: fb[f].data_ptr() + a_lo * fb[f].element_size() for f in FIELDS}
        self._ops = _abi.SmxOps(self.n_a, self.n_b, self.n_sym, fp["kind"], fp["ts"], fp["hi"],
                                fp["lo"], fp["sym"], fp["v0"], fp["v1"], gap)
        self._out = _abi.SmxComposeOut(_ptr(self.order), _ptr(self.addr), _ptr(self.file),
                                       _ptr(self.ctx), _ptr(self.conf), self.cap,
                                       _ptr(self.counts))
        sh = _abi.SmxShard()
        sh.rank, sh.world = self.rank, self.world
        sh.src_a, sh.src_b = self.src_a, self.src_b
        sh.summary = _ptr(self.summary)
        sh.halo_cap = self.H
        sh.export_sym, sh.export_cls, sh.export_src = (_ptr(self.xport[i]) for i in range(3))
        sh.part_tab = _ptr(self.part)
        sh.fin_tab = _ptr(self.part)
        sh.glob = _ptr(self.glob)
        if self.H > 0:
            for b in range(2):
                sh.halo_sym[b], sh.halo_cls[b], sh.halo_src[b] = (_ptr(self.halo[b, i]) for i in range(3))
        sh.halo_dev = _ptr(self.halo_dev)
        sh.in_state_dev = _ptr(self.in_dev)
        sh.src_map = _ptr(self.src_map) if self._map_on else None
        self._sh = sh

    def _step(self, step: int) -> None:
        s = self.torch.cuda.current_stream(self.dev).cuda_stream
        check(lib().smx_shard_step(C.byref(self._ops), C.byref(self._sh), C.byref(self._out),
                                   _ptr(self._ws), self._ws_bytes, s, step))

    # -- 2..5 -------------------------------------------------------------------------
    def _tables(self, summ: Optional[np.ndarray], rescatter: bool, wide: bool = True) -> None:
        """TABLES (+ the lower shards' move tables when a move has a None value, which
        needs the gathered summaries `summ`) and the MAX all_reduce of the partial
        tables and value widths (collective).  rescatter: the records were consumed by
        an earlier TABLES of this step (a WALK re-run) and are bucketed again.  wide:
        64-bit entries; otherwise 32-bit ones (half the all-reduce), which a value too
        wide for them flags in summary[S_TABOVER] (the caller then redoes it wide)."""
        torch = self.torch
        if rescatter:
            self._step(_abi.SHARD_SCATTER)
        n3 = 3 * max(self.n_sym, 1)
        if not wide and self.part32 is not None and summ is None:
            self._sh.tab32 = self.tab_bits
            self._sh.part_tab = self._sh.fin_tab = _ptr(self.part32)
            self._step(_abi.SHARD_TABLES)
            self.part32[n3:].copy_(self.summary[S_WIDTH:S_WIDTH + 3])
            self._mvpre = None
            self._sh.mv_prefix = None
            self.tab32_used += 1
            self.comm.all_reduce_max(self.part32)  # last writers and value widths together
            return
        self._sh.tab32 = 0
        self._sh.part_tab = self._sh.fin_tab = _ptr(self.part)
        self._step(_abi.SHARD_TABLES)
        self.part[n3:].copy_(self.summary[S_WIDTH:S_WIDTH + 3])
        mvpre = None
        if summ is not None and summ[:, S_MVNONE].sum() > 0:
            mv = self.comm.all_gather(self.part[: 2 * self.n_sym])      # [world, 2*n_sym]
            mvpre = mv[: self.rank].max(dim=0).values if self.rank > 0 else torch.zeros_like(mv[0])
            mvpre = mvpre.contiguous()
        self._mvpre = mvpre
        self._sh.mv_prefix = _ptr(mvpre) if mvpre is not None else None
        self.comm.all_reduce_max(self.part)        # last writers and value widths together

    def run(self) -> None:
        """One sharded composition (collective: every rank calls it).  One host sync in
        the pipeline: the exchange's split sizes.  Everything after it -- ORDER, WALK, the
        tables and their all_reduce, EMIT -- is enqueued speculatively, and the gathered
        walk summaries are read once at the end, when the step's work is done; in the
        rare case they call for it (the walk re-ran for a region handed across shards, an
        ORDER failed, a table value was too wide for 32 bits, a move has a None value)
        the tables and EMIT are redone."""
        self.exchange()
        self._step(_abi.SHARD_ORDER)
        self._order_exchange()
        self.in_dev.zero_()
        self._step(_abi.SHARD_WALK)
        self._tables(None, rescatter=False, wide=False)
        self._emit(None)
        summ, reran = self._walk(first_done=True)
        final = (not reran and not summ[:, S_FAIL].any() and summ[:, S_MVNONE].sum() == 0
                 and not summ[:, S_TABOVER].any())
        if summ[:, S_FAIL].any():          # an asynchronous ORDER failed somewhere
            if int(np.bitwise_or.reduce(summ[:, S_FAIL])) & 3:
                self._fail(summ)
            err = None
            if summ[self.rank, S_FAIL]:     # dense timestamp ties: smaller windows, else generic
                self.order_fixes += 1
                try:
                    self._compact()
                    self._step(_abi.SHARD_ORDER_FIX)
                except RuntimeError as e:   # reported by every rank below
                    err = e
            self._order_exchange()
            summ, _ = self._walk()
            if summ[:, S_FAIL].any():
                self._fail(summ, err)
        if not final:  # the speculative tables and EMIT do not hold: every rank redoes them
            self.tab_redo += int(bool(summ[:, S_TABOVER].any()))
            self.emit_redo += 1
            self._tables(summ, rescatter=True)
            self._emit(summ)
        self.sum_walk = summ
        if self.restore:
            self._restore()

    def _emit(self, summ: Optional[np.ndarray]) -> None:
        """EMIT from the gathered summaries, or speculatively (summ None: before they are
        read, as if no move had a None value -- run() redoes it when one has)."""
        if summ is None:
            self._sum_host = np.zeros(self.summary.numel(), np.int64)
        else:
            self._sum_host = np.ascontiguousarray(summ[self.rank], dtype=np.int64)
        self._sh.summary_host = self._sum_host.ctypes.data
        self._step(_abi.SHARD_EMIT)

    def _fail(self, summ: np.ndarray, err=None):
        f = int(np.bitwise_or.reduce(summ[:, S_FAIL]))
        if f & 2:
            raise ValueError("invalid input: sym[i] >= n_sym or kind[i] >= 18")
        raise RuntimeError("sharded merge: the order plan failed on a shard"
                           + (f" ({err})" if err else " (branch logs not timestamp-ordered)"))

    def _order_exchange(self) -> None:
        """One all_gather of every shard's summary and halo exports; the WALK step
        assembles this shard's halo (the first H renames of each branch on the
        following shards) from it on the device (smx_shard.order_gather): no host read."""
        torch = self.torch
        if self.H <= 0:
            self.halo_dev.zero_()
            self._sh.order_gather = None
            return
        self._gathered = self.comm.all_gather(self._sx)
        self._sh.order_gather = _ptr(self._gathered)

    def _walk(self, first_done: bool = False):
        """Walk with the incoming open region of the previous shards (device-held); one
        summary all_gather + host read per round; a shard whose incoming region changed
        re-runs, until none does (a region hand-off moves one shard per round).  Every
        rank sees every summary, so all take the same decisions without another
        collective.  first_done: this step's first WALK is already enqueued.  Returns
        (the gathered summaries, whether any shard re-ran)."""
        W, r = self.world, self.rank
        used = [(0, 0)] * W
        reran = False
        if not first_done:
            self.in_dev.zero_()
            self._step(_abi.SHARD_WALK)
        for _ in range(W + 1):
            summ = self.comm.all_gather(self.summary).cpu().numpy()
            if summ[:, S_FAIL].any():
                break
            if summ[:, S_OVER].any():
                raise AssertionError("sharded walk: a DivergentRename region crosses a shard "
                                     "boundary deeper than the halo (raise halo_cap)")
            want = [(int(summ[q - 1, S_AHEAD]), int(summ[q - 1, S_D]))
                    if q > 0 and summ[q - 1, S_OPEN] else (0, 0) for q in range(W)]
            if want == used:
                break
            reran = True
            if want[r] != used[r]:
                self.in_dev.copy_(self.torch.tensor(want[r], dtype=self.torch.int64))
                self._step(_abi.SHARD_WALK)
            used = want
        self.in_state = used[r]
        return summ, reran

    def totals(self) -> Tuple[int, int]:
        """(composed ops, conflicts) of the whole merge after run() (collective)."""
        g = self.comm.all_gather(self.counts).cpu().numpy()
        return int(g[:, 0].sum()), int(g[:, 1].sum())

    # -- results ----------------------------------------------------------------------
    def results(self):
        """This shard's (order, addr, file, ctx, conflicts) and its kind segments
        [(kind, start, length)] in its local output."""
        torch = self.torch
        torch.cuda.synchronize(self.dev)
        k, nc = (int(x) for x in self.counts.cpu().tolist())
        if k < 0:
            raise RuntimeError("invalid input: sym >= n_sym or kind >= 18")
        if nc > self.cap:
            raise RuntimeError(f"{nc} conflicts exceed capacity {self.cap}")
        kc = self.sum_walk[self.rank, S_KINDS:S_KINDS + N_KINDS].astype(np.int64).copy()
        kc[1] -= int(self.sum_walk[self.rank, S_NSKIP])
        starts = np.concatenate([[0], np.cumsum(kc)])
        segs = [(kk, int(starts[kk]), int(kc[kk])) for kk in range(N_KINDS)]
        return (self.order[:k].cpu().numpy(), self.addr[:k].cpu().numpy(),
                self.file[:k].cpu().numpy(), self.ctx[:k].cpu().numpy(),
                self.conf[: 2 * nc].cpu().numpy().reshape(nc, 2), segs)


def assemble(parts: List[tuple]):
    """Global composed log from every shard's results() (in shard order): kind by kind,
    the shards' segments concatenated; conflicts in shard order."""
    outs = [[], [], [], []]
    for kk in range(N_KINDS):
        for p in parts:
            _, st, ln = p[5][kk]
            for i in range(4):
                outs[i].append(p[i][st:st + ln])
    conf = np.concatenate([p[4] for p in parts]) if parts else np.zeros((0, 2), np.int32)
    return tuple(np.concatenate(o) if o else np.zeros(0, np.int32) for o in outs) + (conf,)
