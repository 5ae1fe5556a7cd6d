/*
 * oracle/compose_ref.c — CPU restatement of the reference composer, for TESTS ONLY.
 *
 * This is the parity checker, never the product: only tests/, the smoke() entry
 * point and bench.py's cpu_baseline leg may load it (libsmx_oracle.so).  It walks
 * the reference algorithm of semmerge/compose.py step for step, on the SoA of
 * include/smx.h with HOST pointers:
 *   sort_key / sorted      compose.py:16-21   (stable per-branch sort)
 *   merge loop             compose.py:51-112  (A on ties, compose.py:54)
 *   DivergentRename skip   compose.py:60-70, 88-98
 *   rename_chain           compose.py:71-72, 99-100
 *   move_chain             compose.py:73-82, 101-110
 *   materialize            compose.py:30-49
 * Pinned against golden vectors produced by the reference itself
 * (tests/golden/, tools/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/smx.h"

static const smx_ops* g_ops; /* qsort has no context argument */

/* (prec, ts, id) then the original position: makes qsort behave like the
 * stable sort of compose.py:20-21. */
static int cmp_key(const void* pa, const void* pb) {
  int64_t a = *(const int64_t*)pa, b = *(const int64_t*)pb;
  const smx_ops* o = g_ops;
  if (o->kind[a] != o->kind[b]) return o->kind[a] < o->kind[b] ? -1 : 1;
  if (o->ts[a] != o->ts[b]) return o->ts[a] < o->ts[b] ? -1 : 1;
  if (o->oid_hi[a] != o->oid_hi[b]) return o->oid_hi[a] < o->oid_hi[b] ? -1 : 1;
  if (o->oid_lo[a] != o->oid_lo[b]) return o->oid_lo[a] < o->oid_lo[b] ? -1 : 1;
  return a < b ? -1 : (a > b);
}

/* sort_key(A) <= sort_key(B) (compose.py:54) */
static int key_le(const smx_ops* o, int64_t a, int64_t b) {
  if (o->kind[a] != o->kind[b]) return o->kind[a] < o->kind[b];
  if (o->ts[a] != o->ts[b]) return o->ts[a] < o->ts[b];
  if (o->oid_hi[a] != o->oid_hi[b]) return o->oid_hi[a] < o->oid_hi[b];
  return o->oid_lo[a] <= o->oid_lo[b];
}

typedef struct {
  int32_t* rename; /* rename_chain[sym]: string id, -1 = absent */
  int32_t* addr;   /* move_chain[sym]["newAddress"], -1 = absent */
  int32_t* file;   /* move_chain[sym]["newFile"], -1 = absent */
} chains;

static int divergent(const smx_ops* o, int64_t a, int64_t b) {
  /* both renames on the same symbol with newName values that are != */
  return o->kind[a] == SMX_KIND_RENAME && o->kind[b] == SMX_KIND_RENAME &&
         o->sym[a] == o->sym[b] && o->v0[a] != o->v0[b];
}

static void take(const smx_ops* o, chains* c, int64_t i) {
  uint32_t s = o->sym[i];
  if (o->kind[i] == SMX_KIND_RENAME) c->rename[s] = o->v1[i];
  if (o->kind[i] == SMX_KIND_MOVE) {
    if (o->v0[i] != SMX_NONE) c->addr[s] = o->v0[i];
    if (o->v1[i] != SMX_NONE) c->file[s] = o->v1[i];
  }
}

static void emit(const smx_ops* o, const chains* c, int64_t i, const smx_compose_out* out,
                 int64_t k) {
  uint32_t s = o->sym[i];
  out->order[k] = (int32_t)i;
  /* Absent chain entries and None values both read as -1: materialize only
   * applies non-None values (compose.py:38-46). */
  out->addr[k] = c->addr[s];
  out->file[k] = c->file[s];
  out->ctx[k] = (o->kind[i] != SMX_KIND_RENAME) ? c->rename[s] : SMX_NONE;
}

int smx_oracle_compose(const smx_ops* o, const smx_compose_out* out) {
  int64_t na = o->n_a, nb = o->n_b;
  int64_t* sa = (int64_t*)malloc(sizeof(int64_t) * (size_t)(na + 1));
  int64_t* sb = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nb + 1));
  chains c;
  size_t ns = (size_t)(o->n_sym > 0 ? o->n_sym : 1);
  c.rename = (int32_t*)malloc(sizeof(int32_t) * ns);
  c.addr = (int32_t*)malloc(sizeof(int32_t) * ns);
  c.file = (int32_t*)malloc(sizeof(int32_t) * ns);
  if (!sa || !sb || !c.rename || !c.addr || !c.file) {
    free(sa); free(sb); free(c.rename); free(c.addr); free(c.file);
    return SMX_E_ARG;
  }
  for (size_t s = 0; s < ns; ++s) c.rename[s] = c.addr[s] = c.file[s] = SMX_NONE;
  for (int64_t i = 0; i < na; ++i) sa[i] = i;
  for (int64_t i = 0; i < nb; ++i) sb[i] = na + i;
  g_ops = o;
  qsort(sa, (size_t)na, sizeof(int64_t), cmp_key);
  qsort(sb, (size_t)nb, sizeof(int64_t), cmp_key);

  int64_t ia = 0, ib = 0, k = 0, nc = 0;
  int rc = SMX_OK;
  while (ia < na || ib < nb) {
    int use_a = ia < na && (ib >= nb || key_le(o, sa[ia], sb[ib]));
    if (ia < na && ib < nb && divergent(o, sa[ia], sb[ib])) {
      /* conflict_divergent_rename(op_a, op_b): always (A, B) order */
      if (nc < out->conflict_cap) {
        out->conflicts[2 * nc] = (int32_t)sa[ia];
        out->conflicts[2 * nc + 1] = (int32_t)sb[ib];
      } else {
        rc = SMX_E_CAPACITY;
      }
      ++nc;
      ++ia;
      ++ib;
      continue;
    }
    int64_t i = use_a ? sa[ia++] : sb[ib++];
    take(o, &c, i);
    emit(o, &c, i, out, k++);
  }
  out->counts[0] = k;
  out->counts[1] = nc;
  free(sa); free(sb); free(c.rename); free(c.addr); free(c.file);
  return rc;
}
