"""Sharded single merge: one composition spread over the GPUs of a node.

The reference composes two branch logs in one sequential loop (semmerge/compose.py:11-114).
Its output order T is (precedence, timestamp, id, side, index): kind-major, so a shard that
owns every op of both branches whose timestamp falls in a key range [tau_r, tau_{r+1}) owns,
for each kind, one contiguous piece of T, and the pieces of the shards follow each other in
shard order.  One process per GPU; the steps of one merge are

1. exchange   each rank starts with an index slice of each branch log (how the logs are
              loaded); one all-to-all (RCCL over xGMI) moves every op to the rank owning its
              timestamp.  Lift-shaped logs are timestamp-ordered, so only the ops near the
              slice edges move.
2. order      smx_shard_step(ORDER): the single-GPU plan + window kernels on the shard.
3. walk       the DivergentRename walk (compose.py:60-70, 88-98) runs per shard; the natural
              head of a rename near a shard's end can be a rename of a later shard, so each
              shard gets a halo (the next renames of each branch, all-gathered), and a region
              still open at a shard's end is handed to the next shard (re-run on the rare
              shards whose incoming region changed).
4. tables     per-symbol last writers (compose.py:27-28, 71-82, 99-110): each shard's
              partial tables tagged (shard + 1) << 32, one MAX all-reduce keeps the last
              writer over shards.
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
N_KINDS = 18


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
        import torch
        x = self._host(t.contiguous())
        out = torch.empty(int(sum(out_splits)), dtype=x.dtype, device=x.device)
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
    return t ^ (-(2 ** 63))


class ShardedCompose:
    """One rank's part of a sharded merge.  `a`, `b`: this rank's index slices of the
    global branch logs (timestamp-ordered), na_glob / nb_glob the global branch sizes.

    The slices are copied once into field buffers with `headroom` free entries on both
    sides of each branch range; the exchange writes the ops arriving from the
    neighbouring shards into the headroom, so the ops that stay (nearly all of them on
    lift-shaped logs) never move, and the shard is handed to the kernels in place:
    A' at [a_lo, a_hi) and B' at [b_lo, b_hi) of every field buffer, B' after a gap
    (smx_ops.b_gap)."""

    def __init__(self, a: BranchSlice, b: BranchSlice, na_glob: int, nb_glob: int, n_sym: int,
                 comm: Comm, device, halo_cap: int = 4096, headroom: Optional[int] = None,
                 restore: bool = True) -> None:
        import torch
        self.torch = torch
        self.na_glob, self.nb_glob = na_glob, nb_glob
        self.n_sym = n_sym
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self.dev = torch.device(device)
        self.H = halo_cap
        self.restore = restore
        self.na_s, self.nb_s = a.n, b.n
        self.a_start, self.b_start = a.start, b.start
        hd = headroom if headroom is not None else max(1 << 16, (a.n + b.n) // 32)
        self._alloc(hd, a, b)
        self._ws = None
        self._ws_bytes = 0
        self._outn = -1
        self.summary = torch.zeros(_abi.SHARD_SUMMARY, dtype=torch.int64, device=self.dev)
        self.xsym = torch.zeros(2 * self.H, dtype=torch.int32, device=self.dev)
        self.xcls = torch.zeros(2 * self.H, dtype=torch.int32, device=self.dev)
        self.xsrc = torch.zeros(2 * self.H, dtype=torch.int32, device=self.dev)
        self.part = torch.zeros(3 * max(n_sym, 1), dtype=torch.int64, device=self.dev)
        self.glob = torch.zeros(3, dtype=torch.int64, device=self.dev)

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

    def _splitters(self) -> np.ndarray:
        """tau[1..world-1]: shard r owns timestamps in [tau[r], tau[r+1])."""
        torch = self.torch
        info = torch.zeros(6, dtype=torch.int64, device=self.dev)
        info[0], info[1] = self.na_s, self.nb_s
        ta, tb = self._orig(0, "ts"), self._orig(1, "ts")
        if self.na_s:
            info[2], info[3] = _u64_key(ta[0]), _u64_key(ta[-1])
        if self.nb_s:
            info[4], info[5] = _u64_key(tb[0]), _u64_key(tb[-1])
        g = self.comm.all_gather(info).cpu().numpy()
        for side, (ni, fi, li) in enumerate(((0, 2, 3), (1, 4, 5))):
            nz = g[g[:, ni] > 0]
            if len(nz) > 1 and np.any(nz[1:, fi] < nz[:-1, li]):
                raise ValueError("sharded merge needs timestamp-ordered branch logs "
                                 f"(branch {'AB'[side]} decreases across rank slices)")
        tau = np.empty(self.world, dtype=np.int64)
        tau[0] = np.iinfo(np.int64).min
        for r in range(1, self.world):
            cand = g[r, 2] if g[r, 0] else (g[r, 4] if g[r, 1] else tau[r - 1])
            tau[r] = max(tau[r - 1], cand)
        return tau

    def exchange(self) -> None:
        """The all-to-all: every op to the shard owning its timestamp (collective)."""
        torch = self.torch
        r, W = self.rank, self.world
        tau = torch.from_numpy(self._splitters()[1:]).to(self.dev)
        counts = []
        for br, n in ((0, self.na_s), (1, self.nb_s)):
            if n:
                cut = torch.searchsorted(_u64_key(self._orig(br, "ts")).contiguous(), tau, right=False)
                edges = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.dev), cut,
                                   torch.full((1,), n, dtype=torch.int64, device=self.dev)])
                counts.append(edges[1:] - edges[:-1])
            else:
                counts.append(torch.zeros(W, dtype=torch.int64, device=self.dev))
        allc = self.comm.all_gather(torch.stack(counts)).cpu().numpy()  # [src, branch, dest]
        send, recv = allc[r], allc[:, :, r]                              # [br, dest], [src, br]
        lo_s, hi_s = send[:, :r].sum(axis=1), send[:, r + 1:].sum(axis=1)
        lo_r, hi_r = recv[:r].sum(axis=0), recv[r + 1:].sum(axis=0)
        need = int(max(0, (lo_r - lo_s).max(), (hi_r - hi_s).max()))
        if need > self.hd:  # skewed slices: grow the headroom (copies the slices once)
            self._alloc(need + (self.na_s + self.nb_s) // 32, None, None)
        first = [int(allc[:, br, :r].sum()) for br in range(2)]
        self.src_a = first[0]
        self.src_b = self.na_glob + first[1]
        # ranges of the shard in the buffers
        n0 = (self.na_s, self.nb_s)
        base = (self._oa, self._ob)
        self.rng = [(base[br] + int(lo_s[br] - lo_r[br]), base[br] + n0[br] - int(hi_s[br] - hi_r[br]))
                    for br in range(2)]
        in_splits = [0 if d == r else int(send[0, d] + send[1, d]) for d in range(W)]
        out_splits = [0 if q == r else int(recv[q, 0] + recv[q, 1]) for q in range(W)]
        self._saved = []
        moving = int(allc.sum()) - sum(int(allc[q, :, q].sum()) for q in range(W))
        if moving:  # the same decision on every rank: the all-to-all is collective
            soff = [np.concatenate([[0], np.cumsum(send[br])]) for br in range(2)]
            roff = np.concatenate([[0], np.cumsum(out_splits)])
            # received pieces of each branch from the lower / higher shards, in shard order
            idx = {}
            for br in range(2):
                for part, qs in (("lo", range(r)), ("hi", range(r + 1, W))):
                    ii = [np.arange(roff[q] + (recv[q, 0] if br else 0),
                                    roff[q] + (recv[q, 0] if br else 0) + recv[q, br]) for q in qs]
                    ii = np.concatenate(ii) if ii else np.zeros(0, np.int64)
                    idx[br, part] = torch.from_numpy(ii.astype(np.int64)).to(self.dev)
            for f in FIELDS:
                pieces = []
                for d in range(W):
                    if d == r:
                        continue
                    for br in range(2):
                        o = self._orig(br, f)
                        pieces.append(o[soff[br][d]: soff[br][d + 1]])
                sendbuf = torch.cat(pieces) if pieces else self.buf[f][:0]
                got = self.comm.all_to_all(sendbuf, in_splits, out_splits)
                for br in range(2):
                    lo, hi = self.rng[br]
                    o0 = base[br]
                    for part, dst0 in (("lo", lo), ("hi", o0 + n0[br] - int(hi_s[br]))):
                        ix = idx[br, part]
                        if ix.numel() == 0:
                            continue
                        if self.restore:  # originals under the arriving ops, put back after the step
                            self._saved.append((f, dst0, self.buf[f][dst0: dst0 + ix.numel()].clone()))
                        self.buf[f][dst0: dst0 + ix.numel()] = got[ix]
        self.n_a = self.rng[0][1] - self.rng[0][0]
        self.n_b = self.rng[1][1] - self.rng[1][0]
        self._bind()

    def _restore(self) -> None:
        for f, at, t in reversed(self._saved):
            self.buf[f][at: at + t.numel()] = t
        self._saved = []

    # -- device structs -----------------------------------------------------------------
    def _bind(self) -> None:
        torch = self.torch
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
        fp = {f: self.buf[f].data_ptr() + a_lo * self.buf[f].element_size() for f in FIELDS}
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
        sh.export_sym, sh.export_cls, sh.export_src = _ptr(self.xsym), _ptr(self.xcls), _ptr(self.xsrc)
        sh.part_tab = _ptr(self.part)
        sh.fin_tab = _ptr(self.part)
        sh.glob = _ptr(self.glob)
        self._sh = sh

    def _step(self, step: int) -> None:
        s = self.torch.cuda.current_stream(self.dev).cuda_stream
        check(lib().smx_shard_step(C.byref(self._ops), C.byref(self._sh), C.byref(self._out),
                                   _ptr(self._ws), self._ws_bytes, s, step))

    # -- 2..5 -------------------------------------------------------------------------
    def run(self) -> None:
        """One sharded composition (collective: every rank calls it)."""
        torch = self.torch
        self.exchange()
        self._step(_abi.SHARD_ORDER)
        summ = self.comm.all_gather(self.summary).cpu().numpy()
        xs = self.comm.all_gather(torch.stack([self.xsym, self.xcls, self.xsrc]))
        self.sum_order = summ
        self._set_halo(summ, xs)
        self._walk()
        self._step(_abi.SHARD_TABLES)
        summ = self.comm.all_gather(self.summary).cpu().numpy()
        self.glob.copy_(torch.from_numpy(summ[:, S_WIDTH:S_WIDTH + 3].max(axis=0)))
        mvpre = None
        if summ[:, S_MVNONE].sum() > 0:
            mv = self.comm.all_gather(self.part[: 2 * self.n_sym])      # [world, 2*n_sym]
            lower = mv[: self.rank]
            mvpre = lower.max(dim=0).values if self.rank > 0 else torch.zeros_like(mv[0])
            mvpre = mvpre.contiguous()
        self._mvpre = mvpre
        self._sh.mv_prefix = _ptr(mvpre) if mvpre is not None else None
        self.comm.all_reduce_max(self.part)
        self._step(_abi.SHARD_EMIT)
        self.sum_final = self.comm.all_gather(self.summary).cpu().numpy()
        if self.restore:
            self._restore()

    def _set_halo(self, summ: np.ndarray, xs) -> None:
        """Halo of branch b: the renames of b on the following shards, first H of them."""
        torch = self.torch
        H, r, W = self.H, self.rank, self.world
        self._halo = []
        for b in range(2):
            pieces, got = [], 0
            rest = int(summ[r + 1:, S_REN + b].sum())
            for q in range(r + 1, W):
                if got >= H:
                    break
                k = min(int(summ[q, S_REN + b]), H, H - got)
                if k:
                    pieces.append(xs[q, :, b * H: b * H + k])
                    got += k
            if pieces:
                h = torch.cat(pieces, dim=1).contiguous()
            else:
                h = torch.zeros((3, 1), dtype=torch.int32, device=self.dev)
            self._halo.append(h)
            self._sh.halo_n[b] = got
            self._sh.halo_more[b] = 1 if rest > got else 0
            self._sh.halo_sym[b] = _ptr(h[0]) if got else None
            self._sh.halo_cls[b] = _ptr(h[1]) if got else None
            self._sh.halo_src[b] = _ptr(h[2]) if got else None

    def _walk(self) -> None:
        """Walk with the incoming open region of the previous shards; a shard whose
        incoming region changed re-runs, until no shard re-runs (at most world rounds:
        a region hand-off moves one shard per round)."""
        W, r = self.world, self.rank
        used = (0, 0)
        self._sh.in_ahead, self._sh.in_d = used
        self._step(_abi.SHARD_WALK)
        for _ in range(W + 1):
            summ = self.comm.all_gather(self.summary).cpu().numpy()
            if summ[:, S_OVER].any():
                raise RuntimeError("sharded walk: a DivergentRename region crosses a shard "
                                   "boundary deeper than the halo (raise halo_cap)")
            want = (int(summ[r - 1, S_AHEAD]), int(summ[r - 1, S_D])) \
                if r > 0 and summ[r - 1, S_OPEN] else (0, 0)
            rerun = want != used
            if rerun:
                used = want
                self._sh.in_ahead, self._sh.in_d = used
                self._step(_abi.SHARD_WALK)
            if not self._any(rerun):
                break
        self.sum_walk = summ
        self.in_state = used

    def _any(self, flag: bool) -> bool:
        t = self.torch.tensor([1 if flag else 0], dtype=self.torch.int64, device=self.dev)
        self.comm.all_reduce_max(t)
        return bool(t.item())

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
        kc = self.sum_order[self.rank, S_KINDS:S_KINDS + N_KINDS].astype(np.int64).copy()
        kc[1] -= int(self.sum_final[self.rank, S_NSKIP])
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
