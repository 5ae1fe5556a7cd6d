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
// Pipeline: stable LSD radix partition of 40-byte event records by list id (LDS-staged,
// coalesced) -> list bounds -> one block per list, in LDS: order by (value, index), one
// sequential replay per value group, survivors ranked by (anchor, t, author, opid,
// index) -> survivor-count scan -> compaction.
#include <string>

#include "smx_scan.h"

#define RGA_TRY(x)                                                                     \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess)                                                              \
      return smx_set_error(SMX_E_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

// Event record, 5 u64 words, grouped by list by the partition below:
//   w0 = anchor << 32 | t' >> 32,  w1 = t' << 32 | author   (t' = t with the sign bit flipped)
//   w2 = opid_hi, w3 = opid_lo                              -> (w0..w3) is the crdt.py:48-57 key order
//   w4 = value << 32 | op << 30 | event index              (index = creation order, the tie-break)
#define RGA_REC 5
#ifndef RGA_ABL
#define RGA_ABL 0  // timing ablations of k_rga_list<256> (wrong results, in bounds): bit0 no
                   // replay, bit1 no survivor sort
#endif
#define RGA_IDX_MASK 0x3fffffffu
#define RGA_SMALL 256   // lists up to this many events: k_rga_list<RGA_SMALL, 256>, one block per list
#define RGA_MID 1536    // ... up to this: k_rga_list<RGA_MID, 512> over the deferred lists; longer: k_rga_big

// Grouping the events by list: a stable LSD radix partition of whole records on the
// list id, 8 bits per pass (one pass up to 256 lists, two up to 65536, ...).  The first
// pass reads the input columns and packs the records; each pass stages a tile in LDS
// in digit order and writes each digit's run of records contiguously, so every byte
// moves in full cache lines.  Stable: each list's events stay in stream order.
#ifndef RR_NT
#define RR_NT 1024                        // scatter workgroup
#endif
#define RR_NW (RR_NT / WAVE)
#ifndef RREC_ITEMS
#define RREC_ITEMS 3
#endif
#define RREC_TILE (RR_NT * RREC_ITEMS)    // 3072 records (120 KB) per block and pass
#define RREC_SEG (RREC_TILE / RR_NW)      // contiguous records per wave
#define RGA_NDIG 256                      // digits per pass
static_assert(RREC_TILE % BLOCK == 0 && RREC_TILE <= 65535, "tile: k_rrec_hist blocks, u16 slots");

__device__ __forceinline__ u32 rga_list_of(const smx_rga_ops& o, i64 i, i32* err) {
  const u32 l = o.list[i];
  if (l >= (u64)o.n_lists || o.op[i] > 2) {
    *err = 1;
    return 0;
  }
  return l;
}

template <bool FIRST>
__global__ void __launch_bounds__(BLOCK) k_rrec_hist(smx_rga_ops o, const u32* __restrict__ keys, int shift,
                                                     u32* __restrict__ hist, i32* __restrict__ err) {
  __shared__ u32 h[RGA_NDIG];
  h[threadIdx.x] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * RREC_TILE;
#pragma unroll
  for (int it = 0; it < RREC_TILE / BLOCK; ++it) {
    const i64 i = base + it * BLOCK + threadIdx.x;
    if (i < o.n_ops) atomicAdd(&h[((FIRST ? rga_list_of(o, i, err) : keys[i]) >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(i64)blockIdx.x * RGA_NDIG + threadIdx.x] = h[threadIdx.x];
}

// One tile per block: wave multisplit of the tile's records by digit (ranks and
// per-wave digit counts), block scan of the digit totals, records staged in LDS in
// digit order, then every digit's run written contiguously (RREC_TILE / 256 records
// per run on average: whole cache lines).  Pass 2+ reads the previous pass's records
// word by word (consecutive lanes, consecutive words) into their staged slots.
template <bool FIRST>
__global__ void __launch_bounds__(RR_NT) k_rrec_scatter(smx_rga_ops o, const u32* __restrict__ kin,
                                                        const u64* __restrict__ rin, u32* __restrict__ kout,
                                                        u64* __restrict__ rout, int shift,
                                                        const u32* __restrict__ offs) {
  __shared__ u64 srec[RREC_TILE * RGA_REC];  // 120 KB
  __shared__ u32 skey[RREC_TILE];
  __shared__ u16 spos[RREC_TILE];            // tile record -> staged slot (pass 2+)
  __shared__ u16 wc[RR_NW][RGA_NDIG];        // per-wave digit counts, then offsets
  __shared__ u32 lstart[RGA_NDIG];
  __shared__ u32 gofs[RGA_NDIG];
  const int t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  const i64 n = o.n_ops, base = (i64)blockIdx.x * RREC_TILE;
  const u32 cnt = (u32)(n - base < RREC_TILE ? n - base : RREC_TILE);
  i32 dummy = 0;
  for (int x = t; x < RR_NW * RGA_NDIG; x += RR_NT) (&wc[0][0])[x] = 0;
  if (t < RGA_NDIG) gofs[t] = offs[(i64)blockIdx.x * RGA_NDIG + t];
  __syncthreads();
  const u64 lt = lanemask_lt();
  u32 key[RREC_ITEMS], dr[RREC_ITEMS];
#pragma unroll
  for (int it = 0; it < RREC_ITEMS; ++it) {
    const i64 i = base + (i64)w * RREC_SEG + it * WAVE + lane;
    const bool valid = i < n;
    key[it] = valid ? (FIRST ? rga_list_of(o, i, &dummy) : kin[i]) : 0u;
    const u32 d = (key[it] >> shift) & 255u;
    const u64 peers = wave_peers<8>(d, valid);
    const u32 before = wc[w][d];
    dr[it] = d | ((before + (u32)__popcll(peers & lt)) << 8);
    if (valid && (peers >> lane) == 1ull) wc[w][d] = (u16)(before + (u32)__popcll(peers));
  }
  __syncthreads();
  if (t < RGA_NDIG) {
    u32 tot = 0;
#pragma unroll
    for (int q = 0; q < RR_NW; ++q) tot += wc[q][t];
    lstart[t] = tot;
  }
  __syncthreads();
  if (t < WAVE) {  // exclusive scan of the 256 digit totals, 4 per lane
    u32 x[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = lstart[4 * t + j];
      sum += x[j];
    }
    u32 run = wave_incl_sum(sum) - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lstart[4 * t + j] = run;
      run += x[j];
    }
  }
  __syncthreads();
  if (t < RGA_NDIG) {
    u32 acc = lstart[t];
#pragma unroll
    for (int q = 0; q < RR_NW; ++q) {
      const u32 c = wc[q][t];
      wc[q][t] = (u16)acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < RREC_ITEMS; ++it) {
    const u32 li = (u32)(w * RREC_SEG + it * WAVE + lane);
    const i64 i = base + li;
    if (i >= n) continue;
    const u32 d = dr[it] & 255u, p = wc[w][d] + (dr[it] >> 8);
    skey[p] = key[it];
    if (FIRST) {
      u64* r = &srec[p * RGA_REC];
      const u64 tt = (u64)o.t[i] ^ 0x8000000000000000ull;
      r[0] = ((u64)o.anchor[i] << 32) | (tt >> 32);
      r[1] = (tt << 32) | o.author[i];
      r[2] = o.opid_hi[i];
      r[3] = o.opid_lo[i];
      const u32 op = o.op[i] > 2 ? 0u : o.op[i];
      r[4] = ((u64)o.value[i] << 32) | (op << 30) | (u32)i;
    } else {
      spos[li] = (u16)p;
    }
  }
  if (!FIRST) {
    __syncthreads();
    const u64* q = rin + (u64)base * RGA_REC;
    for (u32 x = t; x < cnt * RGA_REC; x += RR_NT) {
      const u32 r = x / RGA_REC, k = x - r * RGA_REC;
      srec[spos[r] * RGA_REC + k] = __builtin_nontemporal_load(&q[x]);
    }
  }
  __syncthreads();
  for (u32 p = t; p < cnt; p += RR_NT) {
    const u32 d = (skey[p] >> shift) & 255u;
    kout[gofs[d] + p - lstart[d]] = skey[p];
  }
  for (u32 x = t; x < cnt * RGA_REC; x += RR_NT) {  // word-wise: consecutive lanes, consecutive words
    const u32 p = x / RGA_REC, k = x - p * RGA_REC;
    const u32 d = (skey[p] >> shift) & 255u;
    rout[(u64)(gofs[d] + p - lstart[d]) * RGA_REC + k] = srec[x];
  }
}

// lstart[l] = first sorted position of list l (an empty list starts where the next
// one does); one pass over the sorted list ids.
__global__ void k_rga_bounds(const u32* __restrict__ keys, i64 n, i64 nl, u32* __restrict__ lstart) {
  for (i64 j = (i64)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (i64)gridDim.x * BLOCK) {
    const i64 l = keys[j];
    const i64 lp = j ? (i64)keys[j - 1] : -1;
    for (i64 L = lp + 1; L <= l; ++L) lstart[L] = (u32)j;
    if (j == n - 1)
      for (i64 L = l + 1; L < nl; ++L) lstart[L] = (u32)n;
  }
}

__device__ __forceinline__ u32 rga_lend(const u32* lstart, u32 l, i64 nl, i64 n) {
  return l + 1 < nl ? lstart[l + 1] : (u32)n;
}

// a before b in (key, creation index) order; records as above
__device__ __forceinline__ bool rec_lt(const u64* a, const u64* b) {
  if (a[0] != b[0]) return a[0] < b[0];
  if (a[1] != b[1]) return a[1] < b[1];
  if (a[2] != b[2]) return a[2] < b[2];
  if (a[3] != b[3]) return a[3] < b[3];
  return (u32)a[4] < (u32)b[4];  // index bits (the op bits above them are fixed per index)
}

// Bitonic sort across a 256-thread block, one (key, payload) per thread, ascending by
// key (all-ascending network: the lower index of each pair keeps the minimum).  Stages
// whose pairs lie within a wave exchange through cross-lane permutes; the three
// stages that cross waves go through LDS.
__device__ __forceinline__ void bitonic_block256(u64& key, u32& pay, u64* lk, u32* lp) {
  const u32 i = threadIdx.x;
#pragma unroll
  for (u32 k = 2; k <= 256; k <<= 1) {
#pragma unroll
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      const u32 mask = j == (k >> 1) ? k - 1 : j;
      u64 ok;
      u32 op;
      if (mask < WAVE) {
        ok = __shfl_xor(key, (int)mask);
        op = __shfl_xor(pay, (int)mask);
      } else {
        lk[i] = key;
        lp[i] = pay;
        __syncthreads();
        ok = lk[i ^ mask];
        op = lp[i ^ mask];
        __syncthreads();
      }
      const bool lower = (i & j) == 0;
      if (lower ? ok < key : key < ok) {
        key = ok;
        pay = op;
      }
    }
  }
}

// Lists of at most CAP events, one block each, everything in LDS:
//  1. load the list's records (contiguous);
//  2. order the events by (value, index) — block bitonic sort when CAP == NT == 256,
//     ranking by counting for the larger tier — and let one thread per value group
//     replay the group in stream order (crdt.py:29-43): insert creates a live element,
//     move pops the live element with the smallest (key, index) and creates one,
//     delete tombstones every present element;
//  3. compact the survivors' keys (wave-aggregated) into contiguous LDS columns;
//  4. order them by (key, index) (crdt.py:45-57): CAP == NT == 256: block bitonic sort
//     on word 0, then each run of equal word 0 (rare) is insertion-sorted on the rest
//     of the key and the index; larger tier: rank by counting.  Write (value, index) in
//     list order at the list's range start; scnt[l] = survivors.
// Grid: list l = blockIdx.x when `todo` is null, else a loop over todo[0..*ntodo).
// Longer lists are appended to defer[] for the next kernel.
template <int CAP, int NT>
__global__ void __launch_bounds__(NT) k_rga_list(const u64* __restrict__ R, const u32* __restrict__ lstart, i64 n,
                                                 i64 nl, const u32* __restrict__ todo, const u32* __restrict__ ntodo,
                                                 u32* __restrict__ defer, u32* __restrict__ ndefer,
                                                 u32* __restrict__ tmp_v, u32* __restrict__ tmp_s,
                                                 u32* __restrict__ scnt) {
  constexpr bool SMALL = CAP == 256 && NT == 256;
  __shared__ u64 rec[CAP * RGA_REC];
  // larger tier: (value << 30 | index) by record, then the survivors' words 0 .. 4
  __shared__ u64 gk[SMALL ? 1 : CAP];
  __shared__ u64 sk[4][SMALL ? 1 : CAP];
  __shared__ u16 perm[CAP];              // (value, index) order -> record
  __shared__ u16 surv[SMALL ? CAP : 1];  // SMALL: surviving records
  __shared__ u64 gs[SMALL ? CAP : 1];    // SMALL: (value << 30 | index), sorted
  __shared__ u8 st[CAP];        // bit0 present, bit1 tombstoned (by record, or by (value, index) position)
  __shared__ u64 lk[SMALL ? 256 : 1];
  __shared__ u32 lp[SMALL ? 256 : 1];
  __shared__ u32 ns;
  const u32 t = threadIdx.x, lane = t & (WAVE - 1);
  const u64 lanes_lt = lanemask_lt();
  const u32 nwork = todo ? *ntodo : (u32)gridDim.x;
  for (u32 item = blockIdx.x; item < nwork; item += todo ? gridDim.x : nwork) {
    const u32 l = todo ? todo[item] : item;
    const u32 s0 = lstart[l], cnt = rga_lend(lstart, l, nl, n) - s0;
    if (cnt > (u32)CAP) {
      if (t == 0) defer[atomicAdd(ndefer, 1u)] = l;
      continue;
    }
    __syncthreads();  // the previous list's LDS reads are done
    if (t == 0) ns = 0;
    for (u32 w = t; w < cnt * RGA_REC; w += NT) rec[w] = R[(u64)s0 * RGA_REC + w];
    __syncthreads();
    // survivor: record position when SMALL, else (value, index) position -> perm
    if constexpr (SMALL) {  // (value, index) order by a block bitonic sort; gk, perm by position
      u64 key = ~0ull;
      u32 pay = t;
      if (t < cnt) {
        const u64 w4 = rec[t * RGA_REC + 4];
        key = ((w4 >> 32) << 30) | (w4 & RGA_IDX_MASK);
      }
      bitonic_block256(key, pay, lk, lp);
      gs[t] = key;
      perm[t] = (u16)pay;
      st[t] = 0;
      __syncthreads();
#if RGA_ABL & 1
      if (t < cnt) st[t] = t % 3 != 0;
      if (0)
#endif
      if (t < cnt && (t == 0 || (gs[t - 1] >> 30) != (key >> 30))) {  // group head: replay in stream order
        const u64 v = key >> 30;
        u32 end = t + 1;
        while (end < cnt && (gs[end] >> 30) == v) ++end;
        for (u32 x = t; x < end; ++x) {
          const u32 op = (u32)(rec[perm[x] * RGA_REC + 4] >> 30) & 3u;
          if (op == 2) {
            for (u32 y = t; y < x; ++y)
              if (st[y] & 1) st[y] |= 2;
            continue;  // a delete creates nothing
          }
          if (op == 1) {
            int best = -1;
            for (u32 y = t; y < x; ++y)
              if (st[y] == 1 && (best < 0 || rec_lt(&rec[perm[y] * RGA_REC], &rec[perm[best] * RGA_REC])))
                best = (int)y;
            if (best >= 0) st[best] = 0;
          }
          st[x] = 1;
        }
      }
    } else {
      for (u32 i = t; i < cnt; i += NT) {
        const u64 w4 = rec[i * RGA_REC + 4];
        gk[i] = ((w4 >> 32) << 30) | (w4 & RGA_IDX_MASK);
        st[i] = 0;
      }
      __syncthreads();
      for (u32 i = t; i < cnt; i += NT) {
        const u64 k = gk[i];
        u32 r = 0, j = 0;
        for (; j + 4 <= cnt; j += 4) r += (gk[j] < k) + (gk[j + 1] < k) + (gk[j + 2] < k) + (gk[j + 3] < k);
        for (; j < cnt; ++j) r += gk[j] < k;
        perm[r] = (u16)i;
      }
      __syncthreads();
      for (u32 j = t; j < cnt; j += NT) {
        const u64 v = gk[perm[j]] >> 30;
        if (j != 0 && (gk[perm[j - 1]] >> 30) == v) continue;
        u32 end = j + 1;
        while (end < cnt && (gk[perm[end]] >> 30) == v) ++end;
        for (u32 x = j; x < end; ++x) {
          const u32 op = (u32)(rec[perm[x] * RGA_REC + 4] >> 30) & 3u;
          if (op == 2) {
            for (u32 y = j; y < x; ++y)
              if (st[y] & 1) st[y] |= 2;
            continue;
          }
          if (op == 1) {
            int best = -1;
            for (u32 y = j; y < x; ++y)
              if (st[y] == 1 && (best < 0 || rec_lt(&rec[perm[y] * RGA_REC], &rec[perm[best] * RGA_REC])))
                best = (int)y;
            if (best >= 0) st[best] = 0;
          }
          st[x] = 1;
        }
      }
    }
    __syncthreads();
    for (u32 j0 = 0; j0 < cnt; j0 += NT) {
      const u32 j = j0 + t;
      const bool live = j < cnt && st[j] == 1;
      const u64 ball = __ballot(live);
      u32 got = 0;
      if (lane == 0 && ball) got = atomicAdd(&ns, (u32)__popcll(ball));
      const u32 base = __shfl(got, 0);
      if (live) {
        const u32 a = base + (u32)__popcll(ball & lanes_lt);
        if constexpr (SMALL) {
          surv[a] = perm[j];
        } else {
          const u32 p = perm[j];
          gk[a] = rec[p * RGA_REC];
          sk[0][a] = rec[p * RGA_REC + 1];
          sk[1][a] = rec[p * RGA_REC + 2];
          sk[2][a] = rec[p * RGA_REC + 3];
          sk[3][a] = rec[p * RGA_REC + 4];
        }
      }
    }
    __syncthreads();
    const u32 m = ns;
    if constexpr (SMALL) {
      // survivors a, b (record positions) that tie on word 0: the rest of the key, the index
      auto tail_lt = [&](u32 b, u32 a) {
        const u64* ka = &rec[a * RGA_REC];
        const u64* kb = &rec[b * RGA_REC];
        const u32 ia = (u32)ka[4] & RGA_IDX_MASK, ib = (u32)kb[4] & RGA_IDX_MASK;
        return kb[1] != ka[1] ? kb[1] < ka[1] : kb[2] != ka[2] ? kb[2] < ka[2] : kb[3] != ka[3] ? kb[3] < ka[3] : ib < ia;
      };
      u32 pay = t < m ? surv[t] : 0u;
      u64 key = t < m ? rec[pay * RGA_REC] : ~0ull;
      if (!(RGA_ABL & 2)) bitonic_block256(key, pay, lk, lp);
      lk[t] = key;
      lp[t] = pay;
      __syncthreads();
      if (t < m && t + 1 < m && lk[t + 1] == key && (t == 0 || lk[t - 1] != key)) {
        u32 e = t + 2;  // run [t, e) of equal word 0: insertion sort on the rest
        while (e < m && lk[e] == key) ++e;
        for (u32 x = t + 1; x < e; ++x) {
          const u32 v = lp[x];
          u32 y = x;
          while (y > t && tail_lt(v, lp[y - 1])) {
            lp[y] = lp[y - 1];
            --y;
          }
          lp[y] = v;
        }
      }
      __syncthreads();
      if (t < m) {
        const u64 w4 = rec[lp[t] * RGA_REC + 4];
        tmp_v[s0 + t] = (u32)(w4 >> 32);
        tmp_s[s0 + t] = (u32)w4 & RGA_IDX_MASK;
      }
    } else {
      auto tail_lt = [&](u32 b, u32 a) {
        const u64 a1 = sk[0][a], b1 = sk[0][b], a2 = sk[1][a], b2 = sk[1][b], a3 = sk[2][a], b3 = sk[2][b];
        const u32 ia = (u32)sk[3][a] & RGA_IDX_MASK, ib = (u32)sk[3][b] & RGA_IDX_MASK;
        return b1 != a1 ? b1 < a1 : b2 != a2 ? b2 < a2 : b3 != a3 ? b3 < a3 : ib < ia;
      };
      for (u32 a = t; a < m; a += NT) {
        const u64 k0 = gk[a];
        u32 r = 0;
        for (u32 b = 0; b < m; ++b) {
          const u64 x = gk[b];
          r += x < k0 || (x == k0 && b != a && tail_lt(b, a));
        }
        const u64 w4 = sk[3][a];
        tmp_v[s0 + r] = (u32)(w4 >> 32);
        tmp_s[s0 + r] = (u32)w4 & RGA_IDX_MASK;
      }
    }
    if (t == 0) scnt[l] = m;
  }
}

// Block-wide sort of the record positions p[0..cnt) by `less`, in global memory:
// the bitonic network in its all-ascending form (first stage of each merge compares
// i with its mirror i ^ (k - 1)), so positions past cnt act as +infinity and are
// never touched.
template <typename Less>
__device__ void block_sort_positions(u32* p, u32 cnt, Less less) {
  u32 P = 1;
  while (P < cnt) P <<= 1;
  for (u32 k = 2; k <= P; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      const u32 mask = j == (k >> 1) ? k - 1 : j;
      for (u32 i = threadIdx.x; i < P; i += blockDim.x) {
        const u32 q = i ^ mask;
        if (q > i && q < cnt && less(p[q], p[i])) {
          const u32 x = p[i];
          p[i] = p[q];
          p[q] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Lists longer than RGA_MID: the same replay from global memory, one block per list
// (such lists are rare — a whole file's history in one list).  Per list, in its
// record range: gp = positions sorted by (value, index), bst = state by that order;
// then the survivors' positions sorted by (key, index).
__device__ void rga_big_list(const u64* __restrict__ R, u32 l, const u32* __restrict__ lstart, i64 n, i64 nl,
                             u8* __restrict__ bst, u32* __restrict__ gp, u32* __restrict__ tmp_v,
                             u32* __restrict__ tmp_s, u32* __restrict__ scnt) {
  __shared__ u32 ns;
  const u32 t = threadIdx.x, NT = blockDim.x;
  const u32 s0 = lstart[l], cnt = rga_lend(lstart, l, nl, n) - s0;
  const u64* L = R + (u64)s0 * RGA_REC;
  u8* S = bst + s0;
  u32* G = gp + s0;
  auto gkey = [&](u32 x) { const u64 w = L[x * RGA_REC + 4]; return ((w >> 32) << 30) | (w & RGA_IDX_MASK); };
  for (u32 x = t; x < cnt; x += NT) {
    G[x] = x;
    S[x] = 0;
  }
  __syncthreads();
  block_sort_positions(G, cnt, [&](u32 a, u32 b) { return gkey(a) < gkey(b); });
  for (u32 j = t; j < cnt; j += NT) {
    const u64 v = gkey(G[j]) >> 30;
    if (j != 0 && (gkey(G[j - 1]) >> 30) == v) continue;
    u32 end = j + 1;
    while (end < cnt && (gkey(G[end]) >> 30) == v) ++end;
    for (u32 x = j; x < end; ++x) {
      const u32 op = (u32)(L[G[x] * RGA_REC + 4] >> 30) & 3u;
      if (op == 2) {
        for (u32 y = j; y < x; ++y)
          if (S[y] & 1) S[y] |= 2;
        continue;
      }
      if (op == 1) {
        int best = -1;
        for (u32 y = j; y < x; ++y)
          if (S[y] == 1 && (best < 0 || rec_lt(&L[G[y] * RGA_REC], &L[G[best] * RGA_REC]))) best = (int)y;
        if (best >= 0) S[best] = 0;
      }
      S[x] = 1;
    }
  }
  __syncthreads();
  // survivors' positions to the front of G (their order is fixed by the sort below)
  if (t == 0) {
    u32 w = 0;
    for (u32 j = 0; j < cnt; ++j)
      if (S[j] == 1) G[w++] = G[j];
    ns = w;
  }
  __syncthreads();
  const u32 m = ns;
  block_sort_positions(G, m, [&](u32 a, u32 b) { return rec_lt(&L[a * RGA_REC], &L[b * RGA_REC]); });
  for (u32 j = t; j < m; j += NT) {
    const u64 w4 = L[G[j] * RGA_REC + 4];
    tmp_v[s0 + j] = (u32)(w4 >> 32);
    tmp_s[s0 + j] = (u32)w4 & RGA_IDX_MASK;
  }
  if (t == 0) scnt[l] = m;
}

__global__ void __launch_bounds__(1024) k_rga_big(const u64* __restrict__ R, const u32* __restrict__ lstart, i64 n,
                                                  i64 nl, const u32* __restrict__ todo, const u32* __restrict__ ntodo,
                                                  u8* __restrict__ bst, u32* __restrict__ gp,
                                                  u32* __restrict__ tmp_v, u32* __restrict__ tmp_s,
                                                  u32* __restrict__ scnt) {
  for (u32 item = blockIdx.x; item < *ntodo; item += gridDim.x) {
    __syncthreads();
    rga_big_list(R, todo[item], lstart, n, nl, bst, gp, tmp_v, tmp_s, scnt);
  }
}

// Per list: its survivors, in list order, to their place in the output.
__global__ void k_rga_out(const u32* __restrict__ tmp_v, const u32* __restrict__ tmp_s,
                          const u32* __restrict__ lstart, const u32* __restrict__ scnt, const u32* __restrict__ soff,
                          smx_rga_out out) {
  const u32 l = blockIdx.x;
  const u32 s0 = lstart[l], m = scnt[l], d = soff[l];
  for (u32 x = threadIdx.x; x < m; x += BLOCK) {
    out.out_value[d + x] = tmp_v[s0 + x];
    out.out_src[d + x] = (i32)tmp_s[s0 + x];
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
  size_t off[16];
  size_t total;
};

enum { R_REC, R_REC2, R_KEYS, R_KEYS2, R_RHIST, R_TV, R_TS, R_BST, R_GP, R_DEF1, R_DEF2, R_PART, R_LSTART, R_SCNT, R_SOFF, R_N };

static RgaLayout rga_layout(i64 n, i64 nl) {
  const i64 nn = n > 0 ? n : 1;
  size_t sz[R_N];
  sz[R_REC] = sz[R_REC2] = (size_t)nn * RGA_REC * 8;
  sz[R_KEYS] = sz[R_KEYS2] = sz[R_TV] = sz[R_TS] = sz[R_GP] = (size_t)nn * 4;
  {
    const i64 nblk = SMX_CEIL_DIV(nn, (i64)RREC_TILE);
    sz[R_RHIST] = (size_t)256 * nblk * 4 + hscan_tsum_bytes(nblk, 256) + 260 * 4;
  }
  sz[R_BST] = (size_t)nn;
  sz[R_PART] = SCAN_NB * 8 + 64;  // + error word + totals
  sz[R_LSTART] = sz[R_SCNT] = sz[R_SOFF] = sz[R_DEF1] = sz[R_DEF2] = (size_t)(nl + 1) * 4;
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
  u64* rec = (u64*)(b + L.off[R_REC]);
  u64* rec2 = (u64*)(b + L.off[R_REC2]);
  u32* keys = (u32*)(b + L.off[R_KEYS]);
  u32* keys2 = (u32*)(b + L.off[R_KEYS2]);
  u32* rhist = (u32*)(b + L.off[R_RHIST]);
  u32* tmp_v = (u32*)(b + L.off[R_TV]);
  u32* tmp_s = (u32*)(b + L.off[R_TS]);
  u8* bst = (u8*)(b + L.off[R_BST]);
  u32* gp = (u32*)(b + L.off[R_GP]);
  u32* part = (u32*)(b + L.off[R_PART]);
  i32* err = (i32*)(b + L.off[R_PART] + SCAN_NB * 8);
  u32* totals = (u32*)(err + 2);
  u32* lstart = (u32*)(b + L.off[R_LSTART]);
  u32* scnt = (u32*)(b + L.off[R_SCNT]);
  u32* soff = (u32*)(b + L.off[R_SOFF]);
  u32* def1 = (u32*)(b + L.off[R_DEF1]);
  u32* def2 = (u32*)(b + L.off[R_DEF2]);
  u32* ndef = (u32*)(err + 4);  // two deferred-list counters
  const smx_rga_ops o = *ops;
  const int grid = (int)(SMX_CEIL_DIV(n, (i64)BLOCK) < 8192 ? SMX_CEIL_DIV(n, (i64)BLOCK) : 8192);

  RGA_TRY(hipMemsetAsync(err, 0, 32, st));
  {  // records grouped by list: LSD passes over the list id, ping-pong into rec
    int npass = 1;
    while (npass < 4 && ((u64)(nl - 1) >> (8 * npass)) != 0) ++npass;
    const int nblk = (int)SMX_CEIL_DIV(n, (i64)RREC_TILE);
    u32* tsum = rhist + (size_t)256 * nblk;
    u32* dstart = tsum + hscan_tsum_bytes(nblk, 256) / 4;
    u64* rbuf[2] = {npass % 2 ? rec : rec2, npass % 2 ? rec2 : rec};
    u32* kbuf[2] = {keys, keys2};
    for (int p = 0; p < npass; ++p) {
      if (p == 0)
        hipLaunchKernelGGL(k_rrec_hist<true>, dim3(nblk), dim3(BLOCK), 0, st, o, nullptr, 0, rhist, err);
      else
        hipLaunchKernelGGL(k_rrec_hist<false>, dim3(nblk), dim3(BLOCK), 0, st, o, kbuf[(p - 1) & 1], 8 * p, rhist,
                           err);
      hscan(rhist, nblk, 256u, tsum, dstart, st);
      if (p == 0)
        hipLaunchKernelGGL(k_rrec_scatter<true>, dim3(nblk), dim3(RR_NT), 0, st, o, nullptr, nullptr, kbuf[0],
                           rbuf[0], 0, rhist);
      else
        hipLaunchKernelGGL(k_rrec_scatter<false>, dim3(nblk), dim3(RR_NT), 0, st, o, kbuf[(p - 1) & 1],
                           rbuf[(p - 1) & 1], kbuf[p & 1], rbuf[p & 1], 8 * p, rhist);
    }
    hipLaunchKernelGGL(k_rga_bounds, dim3(grid), dim3(BLOCK), 0, st, kbuf[(npass - 1) & 1], n, nl, lstart);
  }
  hipLaunchKernelGGL((k_rga_list<RGA_SMALL, 256>), dim3(nl), dim3(256), 0, st, rec, lstart, n, nl, nullptr, nullptr,
                     def1, ndef, tmp_v, tmp_s, scnt);
  hipLaunchKernelGGL((k_rga_list<RGA_MID, 512>), dim3(512), dim3(512), 0, st, rec, lstart, n, nl, def1, ndef, def2,
                     ndef + 1, tmp_v, tmp_s, scnt);
  hipLaunchKernelGGL(k_rga_big, dim3(256), dim3(1024), 0, st, rec, lstart, n, nl, def2, ndef + 1, bst, gp, tmp_v,
                     tmp_s, scnt);
  RGA_TRY((scan_excl<OpSum, u32, u32>(scnt, soff, nl, nullptr, part, totals, st)));
  hipLaunchKernelGGL(k_rga_out, dim3(nl), dim3(BLOCK), 0, st, tmp_v, tmp_s, lstart, scnt, soff, *out);
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
