// smx_rga.hip — batched RGA replay on gfx950 (semmerge/crdt.py:23-57), C ABI in include/smx.h.
//
// Exact restatement of the sequential list:
//  * The list is always sorted by (key, creation index): insert places the new
//    element before the first strictly greater key (crdt.py:48-57), so equal
//    keys keep insertion order.
//  * An element's fate depends only on the events of its (list, value):
//    move pops the first live element of that value in list order (= the live
//    one with the smallest (key, index)) and always inserts a new element;
//    delete tombstones every present element of that value (crdt.py:33-43).
//  * materialize = live elements in (key, index) order (crdt.py:45-46).
// Pipeline: stable radix sort of events by (list, value) -> one sequential replay
// per (list, value) group -> per list, survivors ranked by (anchor, t, author,
// opid, index) in LDS -> compaction with per-list offsets.
#include <string>

#include "smx_sort.h"

#define RGA_TRY(x)                                                                     \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess)                                                              \
      return smx_set_error(SMX_E_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

#define RGA_LIST_CAP 2048  // lists up to this many events are ranked in LDS
#define RGA_LDS_KEYS 512   // ... with their survivors' keys in LDS up to this many survivors

struct RgaKey {
  u32 anchor;
  i64 t;
  u32 author;
  u64 hi, lo;
};

__device__ __forceinline__ RgaKey rga_key(const smx_rga_ops& o, u32 i) {
  return RgaKey{o.anchor[i], o.t[i], o.author[i], o.opid_hi[i], o.opid_lo[i]};
}

// (key, index) order: crdt.py:48-57 tuple compare, creation index breaks ties
__device__ __forceinline__ bool rga_lt(const RgaKey& a, u32 ia, const RgaKey& b, u32 ib) {
  if (a.anchor != b.anchor) return a.anchor < b.anchor;
  if (a.t != b.t) return a.t < b.t;
  if (a.author != b.author) return a.author < b.author;
  if (a.hi != b.hi) return a.hi < b.hi;
  if (a.lo != b.lo) return a.lo < b.lo;
  return ia < ib;
}

// Sort records: key = (list, value), value word = event index | op << 30 (the op
// travels through the sort, so the group replay reads no per-event array).
#define RGA_IDX_MASK 0x3fffffffu
__global__ void k_rga_init(smx_rga_ops o, u64* __restrict__ keys, u32* __restrict__ vals, i32* __restrict__ err) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < o.n_ops; i += (i64)gridDim.x * BLOCK) {
    const u32 l = o.list[i];
    const u32 op = o.op[i];
    if (l >= (u64)o.n_lists || op > 2) *err = 1;
    keys[i] = ((u64)(l < (u64)o.n_lists ? l : 0) << 32) | o.value[i];
    vals[i] = (u32)i | ((op > 2 ? 0u : op) << 30);
  }
}

// One thread per (list, value) group (a contiguous range of the sorted events, in
// stream order): replay and mark the fate of every element the group creates.
// state is indexed by sorted position: bit0 present, bit1 tombstoned.
__global__ void k_rga_groups(smx_rga_ops o, const u64* __restrict__ keys, const u32* __restrict__ vals,
                             u8* __restrict__ state) {
  const i64 n = o.n_ops;
  for (i64 j = (i64)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (i64)gridDim.x * BLOCK) {
    if (j != 0 && keys[j - 1] == keys[j]) continue;
    i64 end = j + 1;
    while (end < n && keys[end] == keys[j]) ++end;
    for (i64 x = j; x < end; ++x) {
      const u32 op = vals[x] >> 30;
      if (op == 2) {  // delete: tombstone every present element of the value
        for (i64 y = j; y < x; ++y)
          if (state[y] & 1) state[y] |= 2;
        state[x] = 0;
        continue;
      }
      if (op == 1) {  // move: pop the live element with the smallest (key, index)
        i64 best = -1;
        RgaKey bk{};
        u32 bi = 0;
        for (i64 y = j; y < x; ++y) {
          if (state[y] != 1) continue;
          const u32 e = vals[y] & RGA_IDX_MASK;
          const RgaKey ke = rga_key(o, e);
          if (best < 0 || rga_lt(ke, e, bk, bi)) {
            best = y;
            bk = ke;
            bi = e;
          }
        }
        if (best >= 0) state[best] = 0;
      }
      state[x] = 1;  // insert / move creates a live element
    }
  }
}

// lstart[l] = first sorted position of list l (a list without events starts where
// the next one does); lstart[n_lists] = n.  One pass over the sorted keys.
__global__ void k_rga_bounds(const u64* __restrict__ keys, i64 n, i64 nl, u32* __restrict__ lstart) {
  for (i64 j = (i64)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (i64)gridDim.x * BLOCK) {
    const i64 l = (i64)(keys[j] >> 32);
    const i64 lp = j ? (i64)(keys[j - 1] >> 32) : -1;
    for (i64 L = lp + 1; L <= l; ++L) lstart[L] = (u32)j;
    if (j == n - 1)
      for (i64 L = l + 1; L <= nl; ++L) lstart[L] = (u32)n;
  }
}

// One block per list: rank the list's surviving elements by (key, index) and
// write them, in order, at the start of the list's event range of `tmp`.
__global__ void __launch_bounds__(BLOCK) k_rga_list(smx_rga_ops o, const u32* __restrict__ vals,
                                                    const u8* __restrict__ state, const u32* __restrict__ lstart,
                                                    u32* __restrict__ tmp, u32* __restrict__ scnt) {
  __shared__ u32 sidx[RGA_LIST_CAP];
  __shared__ u64 skey[RGA_LDS_KEYS][4];
  __shared__ u32 ns;
  const u32 l = blockIdx.x;
  const u32 s0 = lstart[l], cnt = lstart[l + 1] - s0;
  if (threadIdx.x == 0) ns = 0;
  __syncthreads();
  if (cnt <= RGA_LIST_CAP) {
    for (u32 x = threadIdx.x; x < cnt; x += BLOCK)
      if (state[s0 + x] == 1) sidx[atomicAdd(&ns, 1u)] = vals[s0 + x] & RGA_IDX_MASK;
    __syncthreads();
    const u32 m = ns;
    if (m <= RGA_LDS_KEYS) {
      // survivors' keys packed once into LDS as four order-preserving words
      // (anchor | t_hi, t_lo | author, opid_hi, opid_lo); every lane then ranks
      // its elements against all of them (same b on all lanes: LDS broadcast)
      for (u32 a = threadIdx.x; a < m; a += BLOCK) {
        const u32 i = sidx[a];
        const u64 tt = (u64)o.t[i] ^ 0x8000000000000000ull;  // signed -> unsigned order
        skey[a][0] = ((u64)o.anchor[i] << 32) | (tt >> 32);
        skey[a][1] = (tt << 32) | o.author[i];
        skey[a][2] = o.opid_hi[i];
        skey[a][3] = o.opid_lo[i];
      }
      __syncthreads();
      for (u32 a = threadIdx.x; a < m; a += BLOCK) {
        const u64 k0 = skey[a][0], k1 = skey[a][1], k2 = skey[a][2], k3 = skey[a][3];
        const u32 ia = sidx[a];
        u32 r = 0;
        for (u32 b = 0; b < m; ++b) {
          const u64 b0 = skey[b][0], b1 = skey[b][1], b2 = skey[b][2], b3 = skey[b][3];
          const bool lt = b0 != k0 ? b0 < k0
                        : b1 != k1 ? b1 < k1
                        : b2 != k2 ? b2 < k2
                        : b3 != k3 ? b3 < k3 : sidx[b] < ia;
          r += lt;
        }
        tmp[s0 + r] = ia;
      }
    } else {
      for (u32 a = threadIdx.x; a < m; a += BLOCK) {
        const u32 ia = sidx[a];
        const RgaKey ka = rga_key(o, ia);
        u32 r = 0;
        for (u32 b = 0; b < m; ++b) {
          const u32 ib = sidx[b];
          r += rga_lt(rga_key(o, ib), ib, ka, ia);
        }
        tmp[s0 + r] = ia;
      }
    }
    if (threadIdx.x == 0) scnt[l] = m;
  } else {
    // large list: rank straight from global memory (quadratic; correct for any size)
    u32 m = 0;
    for (u32 x = 0; x < cnt; ++x) m += state[s0 + x] == 1;
    for (u32 a = threadIdx.x; a < cnt; a += BLOCK) {
      const u32 ia = vals[s0 + a] & RGA_IDX_MASK;
      if (state[s0 + a] != 1) continue;
      const RgaKey ka = rga_key(o, ia);
      u32 r = 0;
      for (u32 b = 0; b < cnt; ++b) {
        const u32 ib = vals[s0 + b] & RGA_IDX_MASK;
        if (state[s0 + b] == 1) r += rga_lt(rga_key(o, ib), ib, ka, ia);
      }
      tmp[s0 + r] = ia;
    }
    if (threadIdx.x == 0) scnt[l] = m;
  }
}

__global__ void k_rga_out(smx_rga_ops o, const u32* __restrict__ tmp, const u32* __restrict__ lstart,
                          const u32* __restrict__ scnt, const u32* __restrict__ soff, smx_rga_out out) {
  const u32 l = blockIdx.x;
  const u32 s0 = lstart[l], m = scnt[l], d = soff[l];
  for (u32 x = threadIdx.x; x < m; x += BLOCK) {
    const u32 i = tmp[s0 + x];
    out.out_value[d + x] = o.value[i];
    out.out_src[d + x] = (i32)i;
  }
  if (threadIdx.x == 0) out.out_offsets[l] = d;
}

__global__ void k_rga_fin(const u32* __restrict__ soff_total, i64 n_lists, smx_rga_out out) {
  out.out_offsets[n_lists] = *soff_total;
  out.counts[0] = *soff_total;
}

static bool o_ok(const smx_rga_ops* o) {
  return o->list && o->op && o->value && o->anchor && o->t && o->author && o->opid_hi && o->opid_lo;
}

struct RgaLayout {
  size_t off[12];
  size_t total;
};

enum { R_KEYS, R_VALS, R_K2, R_V2, R_HIST, R_PART, R_STATE, R_LCNT, R_LSTART, R_SCNT, R_TMP, R_N };

static RgaLayout rga_layout(i64 n, i64 nl) {
  const i64 nn = n > 0 ? n : 1;
  const i64 nblk = SMX_CEIL_DIV(nn, (i64)RADIX_TILE);
  size_t sz[R_N];
  sz[R_KEYS] = sz[R_K2] = (size_t)nn * 8;
  sz[R_VALS] = sz[R_V2] = sz[R_TMP] = (size_t)nn * 4;
  sz[R_HIST] = radix_hist_bytes(nn);
  sz[R_PART] = SCAN_NB * 8 + 64;  // + error word + totals
  sz[R_STATE] = (size_t)nn;
  sz[R_LCNT] = sz[R_LSTART] = sz[R_SCNT] = (size_t)(nl + 1) * 4 * 2;
  RgaLayout L;
  size_t acc = 0;
  for (int i = 0; i < R_N; ++i) {
    L.off[i] = acc;
    acc += (sz[i] + 255) & ~(size_t)255;
  }
  L.total = acc;
  return L;
}

extern "C" int smx_rga_workspace_bytes(int64_t n_ops, int64_t n_lists, size_t* bytes) {
  if (!bytes || n_ops < 0 || n_lists < 0) return SMX_E_ARG;
  *bytes = rga_layout(n_ops, n_lists).total;
  return SMX_OK;
}

static int rga_impl(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb, hipStream_t st) {
  const i64 n = ops->n_ops, nl = ops->n_lists;
  if (n < 0 || nl < 0 || n > (i64)RGA_IDX_MASK || nl >= (i64)0x7fffffff)
    return smx_set_error(SMX_E_ARG, "bad sizes");
  if (!out || !out->out_offsets || !out->counts) return smx_set_error(SMX_E_ARG, "null output");
  if (n == 0) {
    RGA_TRY(hipMemsetAsync(out->out_offsets, 0, (size_t)(nl + 1) * 8, st));
    RGA_TRY(hipMemsetAsync(out->counts, 0, 8, st));
    return SMX_OK;
  }
  if (nl < 1) return smx_set_error(SMX_E_ARG, "n_lists must be >= 1");
  if (!o_ok(ops)) return smx_set_error(SMX_E_ARG, "null input pointer");
  const RgaLayout L = rga_layout(n, nl);
  if (!ws || wsb < L.total)
    return smx_set_error(SMX_E_WORKSPACE, ("workspace too small: need " + std::to_string(L.total)).c_str());
  char* b = (char*)ws;
  u64* keys = (u64*)(b + L.off[R_KEYS]);
  u32* vals = (u32*)(b + L.off[R_VALS]);
  u32* part = (u32*)(b + L.off[R_PART]);
  i32* err = (i32*)(b + L.off[R_PART] + SCAN_NB * 8);
  u32* totals = (u32*)(err + 2);
  u8* state = (u8*)(b + L.off[R_STATE]);
  u32* lcnt = (u32*)(b + L.off[R_LCNT]);
  u32* lstart = (u32*)(b + L.off[R_LSTART]);
  u32* scnt = (u32*)(b + L.off[R_SCNT]);
  u32* soff = scnt + (nl + 1);
  u32* tmp = (u32*)(b + L.off[R_TMP]);
  const smx_rga_ops o = *ops;
  const int grid = (int)(SMX_CEIL_DIV(n, (i64)BLOCK) < 4096 ? SMX_CEIL_DIV(n, (i64)BLOCK) : 4096);

  RGA_TRY(hipMemsetAsync(err, 0, 8, st));
  RGA_TRY(hipMemsetAsync(state, 0, (size_t)n, st));
  hipLaunchKernelGGL(k_rga_init, dim3(grid), dim3(BLOCK), 0, st, o, keys, vals, err);
  // stable LSD radix on (list, value): value bytes then list bytes
  int shifts[8], ns = 0;
  for (int d = 0; d < 4; ++d)
    if (((u64)(n - 1) >> (8 * d)) != 0 || d == 0) shifts[ns++] = 8 * d;  // values are < n_ops
  for (int d = 0; d < 4; ++d)
    if (((u64)(nl - 1) >> (8 * d)) != 0) shifts[ns++] = 32 + 8 * d;
  RadixTemp rt{(u64*)(b + L.off[R_K2]), (u32*)(b + L.off[R_V2]), (u32*)(b + L.off[R_HIST]), part};
  RGA_TRY(radix_sort_pairs(keys, vals, n, shifts, ns, rt, st));
  hipLaunchKernelGGL(k_rga_groups, dim3(grid), dim3(BLOCK), 0, st, o, keys, vals, state);
  hipLaunchKernelGGL(k_rga_bounds, dim3(grid), dim3(BLOCK), 0, st, keys, n, nl, lstart);
  hipLaunchKernelGGL(k_rga_list, dim3(nl), dim3(BLOCK), 0, st, o, vals, state, lstart, tmp, scnt);
  RGA_TRY((scan_excl<OpSum, u32, u32>(scnt, soff, nl, nullptr, part, totals, st)));
  hipLaunchKernelGGL(k_rga_out, dim3(nl), dim3(BLOCK), 0, st, o, tmp, lstart, scnt, soff, *out);
  hipLaunchKernelGGL(k_rga_fin, dim3(1), dim3(1), 0, st, totals, nl, *out);
  RGA_TRY(hipGetLastError());
  i32 herr = 0;
  RGA_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  RGA_TRY(hipStreamSynchronize(st));
  if (herr) return smx_set_error(SMX_E_ARG, "invalid input: list >= n_lists or op > 2");
  return SMX_OK;
}

extern "C" int smx_rga_replay(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb,
                              void* stream) {
  if (!ops) return SMX_E_ARG;
  return rga_impl(ops, out, ws, wsb, (hipStream_t)stream);
}

