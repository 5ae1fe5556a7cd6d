/*
 * oracle/crdt_ref.c — CPU restatement of the reference RGA, for TESTS ONLY.
 *
 * Replays each list's event stream exactly like semmerge/crdt.py:
 *   insert            crdt.py:29-31  (before the first element whose key is greater)
 *   move              crdt.py:33-38  (pop the first live element with the value, then insert)
 *   delete            crdt.py:40-43  (tombstone every element with the value)
 *   materialize       crdt.py:45-46
 *   _find_insert_index crdt.py:48-57 (tuple compare of (anchor, t, author, opid))
 * on the SoA of include/smx.h (host pointers).  O(n^2) per list, like the reference.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/smx.h"

typedef struct {
  uint32_t anchor;
  int64_t t;
  uint32_t author;
  uint64_t hi, lo;
  uint32_t value;
  int32_t src;
  int tomb;
} elem;

static int key_lt(const elem* a, const elem* b) {
  if (a->anchor != b->anchor) return a->anchor < b->anchor;
  if (a->t != b->t) return a->t < b->t;
  if (a->author != b->author) return a->author < b->author;
  if (a->hi != b->hi) return a->hi < b->hi;
  return a->lo < b->lo;
}

static void insert_at(elem* v, int64_t* n, const elem* e) {
  int64_t i = 0;
  while (i < *n && !key_lt(e, &v[i])) ++i;
  memmove(&v[i + 1], &v[i], sizeof(elem) * (size_t)(*n - i));
  v[i] = *e;
  ++*n;
}

int smx_oracle_rga(const smx_rga_ops* o, const smx_rga_out* out) {
  int64_t n = o->n_ops, nl = o->n_lists;
  int64_t* start = (int64_t*)calloc((size_t)(nl + 1), sizeof(int64_t));
  int64_t* fill = (int64_t*)calloc((size_t)(nl + 1), sizeof(int64_t));
  int64_t* byl = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
  elem* buf = (elem*)malloc(sizeof(elem) * (size_t)(n + 1));
  if (!start || !fill || !byl || !buf) {
    free(start); free(fill); free(byl); free(buf);
    return SMX_E_ARG;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (o->list[i] >= (uint64_t)nl) { free(start); free(fill); free(byl); free(buf); return SMX_E_ARG; }
    start[o->list[i] + 1]++;
  }
  for (int64_t l = 0; l < nl; ++l) start[l + 1] += start[l];
  for (int64_t i = 0; i < n; ++i) {
    uint32_t l = o->list[i];
    byl[start[l] + fill[l]++] = i; /* stable: stream order kept per list */
  }
  int64_t k = 0;
  for (int64_t l = 0; l < nl; ++l) {
    int64_t m = 0;
    out->out_offsets[l] = k;
    for (int64_t j = start[l]; j < start[l + 1]; ++j) {
      int64_t i = byl[j];
      elem e = {o->anchor[i], o->t[i], o->author[i], o->opid_hi[i], o->opid_lo[i],
                o->value[i], (int32_t)i, 0};
      if (o->op[i] == 0) {
        insert_at(buf, &m, &e);
      } else if (o->op[i] == 1) {
        for (int64_t q = 0; q < m; ++q) {
          if (!buf[q].tomb && buf[q].value == e.value) {
            memmove(&buf[q], &buf[q + 1], sizeof(elem) * (size_t)(m - q - 1));
            --m;
            break;
          }
        }
        insert_at(buf, &m, &e);
      } else {
        for (int64_t q = 0; q < m; ++q)
          if (buf[q].value == e.value) buf[q].tomb = 1;
      }
    }
    for (int64_t q = 0; q < m; ++q) {
      if (buf[q].tomb) continue;
      out->out_value[k] = buf[q].value;
      out->out_src[k] = buf[q].src;
      ++k;
    }
  }
  out->out_offsets[nl] = k;
  out->counts[0] = k;
  free(start); free(fill); free(byl); free(buf);
  return SMX_OK;
}
