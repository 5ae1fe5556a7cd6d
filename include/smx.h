/*
 * smx.h — C ABI of the MI355X op-log composition library (libsmx.so).
 *
 * Replaces, as a drop-in behind the unchanged Python entry points:
 *   smx_compose   <- semmerge/compose.py:11-114  compose_oplogs(delta_a, delta_b)
 *                    (sort_key/_precedence :16-21,130-149; merge loop :51-112;
 *                     DivergentRename check :60-70,88-98 with conflict.py:34-49;
 *                     rename/move chains :27-28,71-82,99-110; materialize :30-49)
 *   smx_rga_replay <- semmerge/crdt.py:23-57  RGA.insert/move/delete/materialize,
 *                    batched over many independent lists
 *
 * Plain C types only.  All device pointers are HIP device (or managed) memory
 * owned by the caller; the library never allocates: temporary space comes from a
 * caller-provided workspace sized by the *_workspace_bytes queries.  Calls are
 * stream-ordered on `stream` (a hipStream_t passed as void*; NULL = the null
 * stream).  smx_compose performs one stream synchronisation (in smx_compose_finish)
 * to check its plan; read device-side counts only after synchronising the stream.
 *
 * Reentrant: host threads may compose concurrently, each on its own stream and
 * workspace (the library's side stream and fork/join events are kept per caller
 * stream; tests/test_gpu_async.py runs two threads on one GPU).
 *
 * The library keeps no handle to the caller's stream after a call returns, so the
 * stream may be destroyed at any time.
 *
 * Return value: 0 on success, a negative SMX_E* code otherwise; the message is
 * available from smx_last_error() (thread-local).  Nothing aborts the process.
 */
#ifndef SMX_H
#define SMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMX_OK 0
#define SMX_E_ARG (-1)      /* bad argument / shape */
#define SMX_E_CAPACITY (-2) /* an output buffer is too small; required size reported */
#define SMX_E_HIP (-3)      /* a HIP runtime call failed */
#define SMX_E_WORKSPACE (-4) /* workspace too small */

/* Dense precedence ranks (compose.py:130-149; unknown type -> 99 -> rank 17). */
#define SMX_KIND_MOVE 0     /* moveDecl, precedence 10 */
#define SMX_KIND_RENAME 1   /* renameSymbol, precedence 11 */
#define SMX_N_KINDS 18
#define SMX_NONE (-1)

/*
 * One merge's input: ops of branch A (indices [0, n_a)) followed by ops of
 * branch B (indices [n_a, n_a + n_b)), struct-of-arrays, device memory.
 *   kind[i]   precedence rank 0..17 of ops[i].type
 *   ts[i]     order-preserving key of str(provenance["timestamp"])
 *   oid_hi/lo order-preserving 128-bit key of ops[i].id
 *   sym[i]    interned target.symbolId, < n_sym
 *   v0[i]     rename: equality class of params["newName"] (conflict test)
 *             move:   string id of str(params["newAddress"]) or SMX_NONE
 *   v1[i]     rename: string id of str(params["newName"]) (rename chain value)
 *             move:   string id of str(params["newFile"] or params["file"]) or SMX_NONE
 *             other kinds: ignored
 */
typedef struct smx_ops {
  int64_t n_a;
  int64_t n_b;
  int64_t n_sym;
  const uint8_t* kind;
  const uint64_t* ts;
  const uint64_t* oid_hi;
  const uint64_t* oid_lo;
  const uint32_t* sym;
  const int32_t* v0;
  const int32_t* v1;
  /* B op j (j >= n_a) is stored at index j + b_gap of every field array (0: right
   * after A).  A sharded merge keeps headroom between its A and B ranges so its
   * exchange moves only the ops that change shard; smx_compose's generic plan
   * (logs not timestamp-ordered) needs b_gap = 0. */
  int64_t b_gap;
} smx_ops;

/*
 * Composed output, device memory, capacity n_a + n_b for the per-op arrays.
 *   order[k]      source index (into A||B) of the k-th composed op
 *   addr[k]       string id of the move-chain newAddress it sees, or SMX_NONE
 *   file[k]       string id of the move-chain newFile it sees, or SMX_NONE
 *   ctx[k]        string id of its renameContext (non-renames), or SMX_NONE
 *   conflicts     (a_idx, b_idx) pairs in the reference's discovery order;
 *                 capacity conflict_cap pairs (min(n_a, n_b) always suffices)
 *   counts[0]     number of composed ops, counts[1] number of conflicts
 */
typedef struct smx_compose_out {
  int32_t* order;
  int32_t* addr;
  int32_t* file;
  int32_t* ctx;
  int32_t* conflicts;
  int64_t conflict_cap;
  int64_t* counts;
} smx_compose_out;

/* Workspace needed by smx_compose for these sizes. */
int smx_compose_workspace_bytes(int64_t n_a, int64_t n_b, int64_t n_sym, size_t* bytes);

/* Compose one merge on the GPU (see the header comment for semantics).
 * = smx_compose_async followed by smx_compose_finish. */
int smx_compose(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                size_t workspace_bytes, void* stream);

/* The same composition in two halves.  smx_compose_async enqueues the plan for
 * timestamp-ordered branch logs (what lift.ts emits) and every later stage with no
 * host synchronisation, so it can be captured in a hipGraph; after the stream has
 * run it, counts[0] >= 0 means the results are complete, -2 that the logs need
 * another plan and -3 that moves with a None newAddress/newFile still need their
 * prefix fix-up: smx_compose_finish (one stream synchronisation) then completes
 * them.  smx_compose_finish on complete results only checks them. */
int smx_compose_async(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                      size_t workspace_bytes, void* stream);
int smx_compose_finish(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                       size_t workspace_bytes, void* stream);

/* Kept for callers of rounds 3-5 (which cached merge graphs per stream): the library
 * caches none now; returns SMX_OK. */
int smx_release_graphs(void* stream);

/* The order plan the last composition on this thread ran (bench reporting). */
#define SMX_PLAN_PRESORTED 0 /* timestamp-ordered logs: presorted windows */
#define SMX_PLAN_SEGMENTED 1 /* ordered logs with long equal-timestamp groups */
#define SMX_PLAN_RADIX 2     /* unordered logs: radix sort on (ts, oid_hi) */
#define SMX_PLAN_RADIX_LO 3  /* ... and oid_lo (duplicate (ts, oid_hi) pairs) */
#define SMX_PLAN_PRESORTED_WIDE 4 /* ordered logs, groups up to 8192 ops: wide presorted windows */
#define SMX_PLAN_SMALL 5     /* merges of at most 2048 ops (any order): one workgroup, one launch */
int smx_last_plan(void);

/* Merges of at most n ops (clamped to 0..2048; default 2048) run as SMX_PLAN_SMALL, one
 * workgroup and one launch; 0 sends every merge through the window plans.  Process-wide;
 * returns the previous limit. */
int64_t smx_set_small_limit(int64_t n);

/*
 * Sharded single merge: one process per GPU, shard r of G.
 * Replaces the same reference loop as smx_compose (compose.py:11-114) for a merge
 * too large for one GPU.  Shard r holds, for both branches, the ops whose
 * timestamp keys fall in its key range [tau_r, tau_{r+1}): contiguous index
 * ranges of the global branch logs (branch logs must be timestamp-ordered, as
 * lift.ts emits them; the host's all-to-all puts them there).  For each kind
 * the shards' T-ordered segments follow each other in shard order, so the
 * global composed log is, kind by kind, the shards' outputs concatenated.
 *
 * The host drives four steps on the same workspace, exchanging the small
 * per-shard summaries (and the partial tables) between them with collectives:
 *   SMX_SHARD_ORDER   plan + window kernels; writes summary[0..21] and the
 *                     first halo_cap renames of each branch (export_*).  With
 *                     src_map == NULL it is asynchronous (no host sync): the
 *                     presorted plan only; a failure shows in summary[21]
 *                     (bit 0 not ordered, bit 1 invalid input, bit 2 a window
 *                     overflowed on dense timestamp ties) and is repaired by
 *   SMX_SHARD_ORDER_FIX  the plan fallbacks (smaller windows; with b_gap = 0 the
 *                     segmented or radix plan, never for a slice whose timestamps
 *                     decrease: that returns SMX_E_ARG); rewrites summary[0..21]
 *                     and the exports
 *   SMX_SHARD_WALK    DivergentRename walk with the halo (the next shards'
 *                     exports) and an incoming open region (in_ahead, in_d);
 *                     may be re-run when the incoming region changes;
 *                     writes summary[22..27]
 *   SMX_SHARD_TABLES  this shard's last writers -> part_tab (MAX-reduce them
 *                     over shards next); writes summary[28..30].  ORDER and
 *                     ORDER_FIX already bucket the table records (beside the
 *                     walk); TABLES applies the walk's skips to them, which it can
 *                     do once (a second TABLES without ORDER / ORDER_FIX / SCATTER
 *                     in between returns SMX_E_ARG):
 *   SMX_SHARD_SCATTER re-buckets the records, for a TABLES after a WALK re-run
 *   SMX_SHARD_EMIT    composed output from the reduced tables (fin_tab) and
 *                     the global value widths (glob[0..2]); mv_prefix (or NULL
 *                     when no move has a None value) = [2][n_sym] last non-None
 *                     move values of the lower shards.  With summary_host set
 *                     (this shard's summary as the host last gathered it) the
 *                     step needs no host sync.
 * Source indices in order[] and conflicts are global: local A op j is
 * src_a + j, local B op j is src_b + j.  summary (int64):
 *   [0..17] ops per kind  [18..19] renames of A, B  [20] moves with a None value
 *   [21] plan failure (not timestamp-ordered / invalid input)
 *   [22] outgoing region open  [23] its ahead branch  [24] its d
 *   [25] conflicts  [26] skipped renames  [27] halo too short
 *   [28..30] bit widths of (value + 1) for addr, file, ctx
 *   [31] a value too wide for the tab32 entries (TABLES with tab32 > 0)
 */
#define SMX_SHARD_ORDER 0
#define SMX_SHARD_WALK 1
#define SMX_SHARD_TABLES 2
#define SMX_SHARD_EMIT 3
#define SMX_SHARD_ORDER_FIX 4
#define SMX_SHARD_SCATTER 5
#define SMX_SHARD_SUMMARY 32

typedef struct smx_shard {
  int32_t rank;
  int32_t world;
  int64_t src_a;
  int64_t src_b;
  /* walk: the renames of each branch after this shard's (device) */
  int64_t halo_n[2];
  int32_t halo_more[2];
  const uint32_t* halo_sym[2];
  const int32_t* halo_cls[2];
  const int32_t* halo_src[2];
  int32_t in_ahead;
  int64_t in_d;
  /* outputs of the steps (device) */
  int64_t* summary;
  int64_t halo_cap;
  uint32_t* export_sym; /* [2][halo_cap] */
  int32_t* export_cls;
  int32_t* export_src;
  uint64_t* part_tab;   /* [3][n_sym] */
  /* inputs of the emit step (device) */
  const uint64_t* fin_tab;   /* [3][n_sym], MAX-reduced part_tab */
  const int64_t* glob;       /* [3] value bit widths, MAX over shards */
  const uint64_t* mv_prefix; /* [2][n_sym] or NULL */
  /* Device-held alternatives, so a step needs no host round trip (NULL: the host
   * fields above are used). */
  const int64_t* halo_dev;     /* [4] halo_n[0], halo_n[1], halo_more[0], halo_more[1] */
  const int64_t* in_state_dev; /* [2] in_ahead, in_d */
  /* A shard built by a sample-sort exchange (branch logs in any order; b_gap = 0):
   * the global source index of each local op j, [n_a + n_b]; replaces src_a/src_b
   * and lets the ORDER step use the generic (sorting) plan.  NULL otherwise. */
  const int32_t* src_map;
  /* host memory: this shard's summary [SMX_SHARD_SUMMARY] after WALK, or NULL */
  const int64_t* summary_host;
  /* Device, or NULL: the all-gather of every shard's ORDER outputs, row q =
   * shard q's summary [SMX_SHARD_SUMMARY] then its exports (export_sym, export_cls,
   * export_src, each [2][halo_cap] 32-bit) -- [world][SMX_SHARD_SUMMARY + 3 * halo_cap]
   * int64.  When set, the WALK step first assembles this shard's halo from it on the
   * device: halo_sym / halo_cls / halo_src ([halo_cap] each, writable) and halo_dev
   * (writable) are then outputs, so the host needs no read of the summaries. */
  const int64_t* order_gather;
  /* 0: part_tab / fin_tab are uint64 [3][n_sym] (+ glob, int64 [3]), entries
   * (rank + 1) << 32 | (value + 1).  tab32 > 0: half the MAX all-reduce -- they are
   * int32 [3 * n_sym + 3], entries (rank + 1) << (31 - tab32) | (value + 1) (a tag of
   * tab32 bits under a clear sign bit, so an int32 MAX keeps the last writer), the
   * three value widths after them (glob unused); a value too wide for the 31 - tab32
   * bits sets summary[31] and the caller redoes the step with tab32 = 0. */
  int32_t tab32;
} smx_shard;

int smx_shard_step(const smx_ops* ops, const smx_shard* shard, const smx_compose_out* out,
                   void* workspace, size_t workspace_bytes, void* stream, int step);

/*
 * The range plan's per-rank info for the sharded exchange (shard.py _range_info), in
 * two launches instead of a dozen tensor operations.  ts: the rank's timestamp buffer;
 * its A slice is ts[off_a, off_a + n_a), its B slice ts[off_b, off_b + n_b).  out
 * (int64, 9 + 4 * rh, device): n_a, n_b; the first and last key of the A slice, of the B
 * slice (keys: the u64 timestamp with its top bit flipped, so that int64 order is u64
 * order; 0 for an empty slice); 1 if both slices are non-decreasing (check_order = 0:
 * not checked, 1); signed_a, signed_b; then rh keys from the head of the A slice and rh
 * from its tail (right-aligned), the same for B (a slice shorter than rh pads with its
 * first key).
 */
int smx_shard_range_info(const uint64_t* ts, int64_t off_a, int64_t n_a, int64_t off_b, int64_t n_b, int32_t rh,
                         int32_t check_order, int32_t signed_a, int32_t signed_b, int64_t* out, void* stream);

/*
 * Per-stage device timing of the last smx_compose calls on this thread, for the
 * benchmark: when enabled, each stage is bracketed by hipEvents on the call's
 * stream and the elapsed milliseconds are accumulated per stage.
 * smx_stage_times copies up to `cap` entries and returns the number of stages;
 * smx_stage_name(i) names stage i.  smx_set_profiling_stages limits the timing to the
 * stages whose bit (1 << i) is set (default: all), so that a benchmark can time one
 * kernel without an event pair around every stage of every merge.
 */
int smx_set_profiling(int enabled);
int smx_set_profiling_stages(uint32_t mask);
int smx_stage_times(double* ms, int64_t* calls, int cap);
const char* smx_stage_name(int i);
int smx_reset_stage_times(void);

/*
 * Batched RGA replay (crdt.py:23-57): n_ops events over n_lists independent
 * lists, events of one list in stream order (list[i] non-decreasing is NOT
 * required; stream order is the index order).
 *   list[i]   list id < n_lists
 *   op[i]     0 = insert(key, value), 1 = move(value, key), 2 = delete(value)
 *   value[i]  interned value (equality class of the value string)
 *   key_*[i]  order-preserving image of Key(anchor, t, author, opid):
 *             anchor rank (u32), t (i64, compared signed), author rank (u32),
 *             opid 128-bit key; ignored for delete
 * Output: out_value[k] for the surviving elements of every list in list order
 * then list-position order, out_offsets[l] = first output index of list l
 * (n_lists + 1 entries), out_src[k] = index of the event that created element k.
 */
typedef struct smx_rga_ops {
  int64_t n_ops;
  int64_t n_lists;
  const uint32_t* list;
  const uint8_t* op;
  const uint32_t* value;
  const uint32_t* anchor;
  const int64_t* t;
  const uint32_t* author;
  const uint64_t* opid_hi;
  const uint64_t* opid_lo;
} smx_rga_ops;

typedef struct smx_rga_out {
  uint32_t* out_value;
  int32_t* out_src;
  int64_t* out_offsets;
  int64_t* counts; /* counts[0] = surviving elements */
  /* NULL: the output is materialize() (live elements only).  Non-NULL: the output is
   * the whole list state RGA.list (crdt.py:26-27) -- the live elements and the ones
   * delete() tombstoned, in list order -- and out_tomb[k] = 1 marks the tombstoned
   * ones (0 the live ones); counts[0] = elements in the lists. */
  uint8_t* out_tomb;
} smx_rga_out;

int smx_rga_workspace_bytes(int64_t n_ops, int64_t n_lists, size_t* bytes);
int smx_rga_replay(const smx_rga_ops* ops, const smx_rga_out* out, void* workspace,
                   size_t workspace_bytes, void* stream);

/* smx_rga_replay with flags.  SMX_RGA_GROUPED: the caller's events come list by list
 * (list ids never decrease -- what crdt.replay and the RGA drop-in build, one stream
 * after another), so the library packs the records in place instead of partitioning
 * them by list.  The claim is checked on the device: a list id that decreases makes the
 * call redo itself through the partition (same results, the partition's cost).
 * smx_rga_replay(...) == smx_rga_replay_ex(..., 0, stream). */
#define SMX_RGA_GROUPED 1u
int smx_rga_replay_ex(const smx_rga_ops* ops, const smx_rga_out* out, void* workspace,
                      size_t workspace_bytes, uint32_t flags, void* stream);

const char* smx_last_error(void);
const char* smx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SMX_H */
