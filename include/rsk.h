/*
 * rsk.h — C ABI of librsk.so, the MI355X (gfx950) placement-scoring library.
 *
 * The reference (ye0nj00/Kubernetes-Rescheduling) is pure Python: its
 * placement policies are the five functions of rescheduling.py and there is no
 * FFI.  This header is the boundary the drop-in Python module
 * (kubernetes-rescheduling_amd/rescheduling.py) binds with ctypes; each entry
 * point names the reference code it replaces.  No torch types cross it: only
 * plain pointers, sizes and status codes.
 *
 * Conventions
 *  - Every pointer argument is caller-owned.  With RSK_F_DEVICE in `flags`,
 *    ALL array pointers of the call are device (HBM) pointers and the call is
 *    asynchronous on the context's stream; otherwise they are host pointers
 *    and the call is synchronous (inputs copied in, outputs copied back).
 *  - Per-scenario arrays are scenario-minor: x[i*S + s] for pod/node/row i and
 *    scenario s.  Per-node constants (cap_cpu, name_rank) are x[n].
 *  - Placement results: >= 0 node index; RSK_TARGET_NONE (-1) where the
 *    reference yields nodeName=None; RSK_TARGET_NO_CANDIDATE (-2) where it raises
 *    (ValueError in communication(), RuntimeError in spread/binpack/random).
 *  - Values: cap_cpu / use_cpu are millicores in [0, 2^31-1]; node indices in
 *    [0, N); an assign entry outside [0, N) means "not on any node".
 *  - Return codes below; rsk_last_error() gives a thread-local message.
 *  - One context = one device + one stream.  A context is not shareable across
 *    threads; separate contexts may run concurrently.
 */
#ifndef RSK_H
#define RSK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSK_OK 0
#define RSK_NO_CANDIDATE 1 /* some cell had no candidate node (host-pointer calls) */
#define RSK_EINVAL 2       /* bad argument: null pointer, size or range */
#define RSK_EHIP 3         /* HIP runtime error */
#define RSK_ERCCL 4        /* reserved: collective error */

#define RSK_F_DEVICE 1u    /* all array pointers are device pointers; async */
#define RSK_F_TILED 4u     /* rsk_car_plan_execute: the tile / side kernels even for a small batch
                              (S <= 4, Q*S <= 65536, no scores), which otherwise runs in one launch */

#define RSK_TARGET_NONE (-1)
#define RSK_TARGET_NO_CANDIDATE (-2)

typedef struct rsk_ctx rsk_ctx;
typedef struct rsk_car_plan rsk_car_plan;
typedef struct rsk_rounds rsk_rounds;

/* ---- library / context ---------------------------------------------------- */
int rsk_version(void);                                /* 100*major + minor */
/* Self-check of the library's u64 workspace layouts for N nodes, S scenarios
 * and a move table of H slots (host arithmetic only, no device): RSK_OK, or
 * RSK_EINVAL with rsk_last_error() naming the first u64 slice whose byte
 * offset is not a multiple of 8.  Every entry point that uses such a layout
 * runs the same check before launching (a misaligned 64-bit atomic faults the
 * GPU, DESIGN.md §6 "r04p2"). */
int rsk_check_ws_layout(int32_t N, int32_t S, int32_t H);
const char *rsk_last_error(void);                     /* thread-local, never NULL */
int rsk_ctx_create(int device, rsk_ctx **out);
int rsk_ctx_destroy(rsk_ctx *ctx);
/* Run subsequent work on `hip_stream` (a hipStream_t; NULL = the context's own). */
int rsk_ctx_set_stream(rsk_ctx *ctx, void *hip_stream);
int rsk_ctx_synchronize(rsk_ctx *ctx);
/* Kernel timing with HIP events recorded on the stream of every launch of the
 * named kernel group: "car_prep" (the node-code pass), "car_tile" (the tile
 * launch, with the side rows fused into it),
 * "car_direct" (a small batch's one launch), "car_side" (side rows launched
 * on their own, e.g. config 4's rows beyond the fused grid on the side stream),
 * "car_mid" / "car_heavy" (the wide path's 33..64 and hub rows, N > 65535),
 * "node_reduce", "load_std", "cut_cost", "rounds_*", ... */
int rsk_ctx_set_profiling(rsk_ctx *ctx, int on);
/* Restrict the timing events to launches of one kernel name (NULL or "" = all):
 * fewer events inside a timed region. */
int rsk_ctx_set_profile_only(rsk_ctx *ctx, const char *kernel);
int rsk_ctx_kernel_time(rsk_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches);
int rsk_ctx_reset_profiling(rsk_ctx *ctx);

/* ---- CAR (communication-aware rescheduling) -------------------------------
 * Replaces the score loop and argmax of `communication`
 * (rescheduling.py:183-214) for a batch of moving pods x scenarios.
 *   row_ptr[P+1], col_idx[nnz] : pod->pod relation CSR: q in row p iff
 *        dep(q) in relations[dep(p)] (main.py:31-52 at pod level).  Host
 *        pointers.  Duplicates and the self edge are dropped by the plan (the
 *        evicted pod is off the cluster, main.py:73).
 *   rows[Q] : the moving pods (NULL = all P, Q ignored).  Host pointer.
 * A plan uploads the CSR once and bins rows by degree; execute() may then run
 * any number of scenario batches against it.                                  */
int rsk_car_plan_create(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                        const int32_t *rows, int32_t Q, rsk_car_plan **out);
int rsk_car_plan_destroy(rsk_car_plan *plan);
/*   assign[P*S], use_cpu[N*S], hazard[N*S] (0/1), cap_cpu[N]
 *   out_target[Q*S] : node per (row, scenario), codes as above
 *   out_score[Q*S]  : max_score of rescheduling.py:199, -1 when no candidate
 *                     (may be NULL)                                            */
int rsk_car_plan_execute(rsk_car_plan *plan, const int32_t *assign, int32_t S, const int32_t *cap_cpu,
                         const int32_t *use_cpu, const uint8_t *hazard, int32_t N,
                         int32_t *out_target, int32_t *out_score, uint32_t flags);
/* Plan layout statistics (host, no GPU work): how the rows were routed.
 * out[0] rows scored in tiles (deg <= 32)   out[1] (unused, 0)
 * out[2] rows of degree 33..64, out[3] rows of degree 65..4096 (the wide
 *        path's car_mid / car_hub classes; the compact path scores both with
 *        car_side16 and counts them in out[15])   out[4] tiles
 * out[5] max image rows per tile   out[6] max owner rows per tile
 * out[7] tile plan bytes   out[8] (unused, 0)   out[9] mid record bytes
 * out[10] hub item + CSR bytes   out[11] max row degree
 * out[12] image rows over all tiles   out[13] distinct pods in the images
 * out[14] rows on the sorted tile class (17..32)   out[15] side rows (> 32)
 * out[16] side item + neighbour bytes   out[17] light_max (tile degree bound)
 * out[18] rows in lean tiles   out[19] lean tiles
 * out[20] side rows the last execute ran inside the lean tile launch
 * out[21] distinct neighbour pods of the tile rows and those side rows
 * out[22] distinct neighbour pods of every row.
 * Returns the number of fields written (<= n).                             */
int rsk_car_plan_info(const rsk_car_plan *plan, int64_t *out, int n);
/* One-shot convenience: plan_create + execute + destroy. */
int rsk_car_place(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                  const int32_t *assign, int32_t S, const int32_t *cap_cpu, const int32_t *use_cpu,
                  const uint8_t *hazard, int32_t N, const int32_t *rows, int32_t Q,
                  int32_t *out_target, int32_t *out_score, uint32_t flags);
/* One CAR placement (S = 1) in one launch, for the drop-in's single call
 * (rescheduling.py:174-218): node_of[k] = the node of each related pod (its
 * neighbours, outside [0, N) ignored); score[n] = #{i : node_of[i] = n} over
 * non-hazard n, then the argmax with the reference's tie-breaks, None (-1)
 * and RSK_NO_CANDIDATE when every node is hazard.  No plan; N <= 32768. */
int rsk_car_row(rsk_ctx *ctx, const int32_t *node_of, int32_t k, const int32_t *cap_cpu, const int32_t *use_cpu,
                const uint8_t *hazard, int32_t N, int32_t *out_target, int32_t *out_score, uint32_t flags);

/* ---- baselines --------------------------------------------------------------
 * spread  (rescheduling.py:89-101): argmin over non-hazard n of
 *         (pod_count[n*S+s], name_rank[n]) -> out_node[s].
 * binpack (rescheduling.py:121-133): argmax of (cpu_pct[n*S+s], name_rank[n]).
 * name_rank[n] = rank of node n's name in Python str (code point) order.      */
int rsk_spread_place(rsk_ctx *ctx, const int32_t *pod_count, const int32_t *name_rank,
                     const uint8_t *hazard, int32_t N, int32_t S, int32_t *out_node, uint32_t flags);
int rsk_binpack_place(rsk_ctx *ctx, const int32_t *cpu_pct, const int32_t *name_rank,
                      const uint8_t *hazard, int32_t N, int32_t S, int32_t *out_node, uint32_t flags);
/* random (rescheduling.py:149-153) in two halves around the caller's RNG:
 *   rsk_random_count:  out_count[s] = #non-hazard nodes (len(candidates))
 *   rsk_random_select: out_node[s] = the r[s]-th non-hazard node in index order
 *                      (candidates[r]); -2 when r is out of range.
 * rsk_random_place draws r[s] = Random(seeds[s])._randbelow(count[s]) with a
 * CPython-compatible MT19937 on the host and runs both halves.               */
int rsk_random_count(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, int32_t *out_count,
                     uint32_t flags);
int rsk_random_select(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, const int32_t *r,
                      int32_t *out_node, uint32_t flags);
/* random's candidate list for the drop-in's single call (S = 1, host
 * pointers; rescheduling.py:149-150): out_nodes[0 .. *out_count) = the
 * non-hazard nodes in index order (nodes_name order), in one launch; the
 * caller draws r = rd.choice(range(count)) and takes out_nodes[r]
 * (rescheduling.py:153).  out_nodes holds N entries. */
int rsk_random_candidates(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t *out_nodes, int32_t *out_count);
int rsk_random_place(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, const uint64_t *seeds,
                     int32_t *out_node, uint32_t flags);
/* CPython random.Random(seed)._randbelow(n) (host only; 0 < n < 2^31). */
int32_t rsk_py_randbelow(uint64_t seed, int32_t n);

/* ---- per-node reductions and metrics (kernel 3) ---------------------------
 * rsk_node_reduce: pod_count[N*S], cpu_sum[N*S], mem_sum[N*S] (NULL to skip)
 *                  of the pods assigned to each (node, scenario).
 * rsk_cpu_pct:     int(round(use / cap * 100)), -1 if cap == 0
 *                  (get_resource_usage.py:37), fp64, round-half-even.
 * rsk_detect:      hazard = pct >= threshold, most[s] = first max hazard node
 *                  or -1 (harzard_detect.py:3-27).
 * rsk_load_std:    population std of use/cap*100 over nodes with cap > 0,
 *                  0.0 if none (nodemonitor.py:24-50); fp64.
 * rsk_cut_cost:    directed count of related pairs on different nodes
 *                  (communicationcost.py:37-45), unscheduled = -1 compares as
 *                  None; missing[p] (may be NULL) adds relations to absent
 *                  deployments.  The reference's cost is out_directed / 2.
 * rsk_pick_max_pod: first pod with the largest pod_cpu on node most[s]
 *                  (delete_replaced_pod.py:41-61), -1 if none.              */
int rsk_node_reduce(rsk_ctx *ctx, const int32_t *assign, int32_t P, int32_t S, const int32_t *pod_cpu,
                    const int64_t *pod_mem, int32_t N, int32_t *pod_count, int64_t *cpu_sum,
                    int64_t *mem_sum, uint32_t flags);
/* Device write guards (DESIGN.md §6 "r05v"): launches whose write offsets
 * come from an earlier launch's counts check them against their buffer and,
 * on overflow, skip the store and set the context's device error word; the
 * context's next entry point (a host-pointer call: its own completion) and
 * rsk_ctx_synchronize return RSK_EHIP naming the kernel.
 * rsk_selftest_write_guard runs rsk_node_reduce on a small internal batch with
 * nr_place's record capacity lowered below its pod count: it returns RSK_EHIP
 * with rsk_last_error() naming nr_place when the guard works, RSK_EINVAL when
 * it did not fire (test hook; no caller data). */
int rsk_selftest_write_guard(rsk_ctx *ctx);
int rsk_cpu_pct(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S,
                int32_t *out_pct, uint32_t flags);
int rsk_detect(rsk_ctx *ctx, const int32_t *cpu_pct, int32_t N, int32_t S, int32_t threshold,
               uint8_t *out_hazard, int32_t *out_most, uint32_t flags);
int rsk_load_std(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S,
                 double *out_std, uint32_t flags);
int rsk_cut_cost(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                 const int32_t *assign, int32_t S, const int32_t *missing, int64_t *out_directed,
                 uint32_t flags);
int rsk_pick_max_pod(rsk_ctx *ctx, const int32_t *assign, const int32_t *pod_cpu, int32_t P, int32_t S,
                     const int32_t *most, int32_t *out_pod, uint32_t flags);
/* rsk_cut_cost over rows [r0, r1) only (pod-row sharding, SURVEY §8e: each
 * rank's partial of communicationcost.py:37-45; neighbours read from the full
 * assign).  row_ptr / col_idx / assign are the full P-row arrays.            */
int rsk_cut_cost_rows(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, int32_t r0,
                      int32_t r1, const int32_t *assign, int32_t S, const int32_t *missing,
                      int64_t *out_directed, uint32_t flags);

/* ---- multi-round loop --------------------
 * The reference's control loop (main.py:55-110) for S independent scenarios,
 * R rounds, all on the device.  Round r, scenario s:
 *   pct = cpu_pct(use, cap) (a9); hazard = pct >= threshold and most = first
 *   max hazard node (a8); p = pick_max_pod(assign, pod_cpu, most) (a10);
 *   t = the CAR target of p (a1/a2) against the round's assign / use / hazard;
 *   then the build-defined update (the reference re-measures the live cluster
 *   instead): when t >= 0 the pod's CPU moves with it, use[old] -= pod_cpu[p],
 *   use[t] += pod_cpu[p], assign[p] = t.  Otherwise the state stays.
 *   out_evict[r*S+s]  = p, -1 when there is no hazard node or no pod on it
 *   out_target[r*S+s] = t: node, RSK_TARGET_NONE, RSK_TARGET_NO_CANDIDATE, or
 *                       RSK_TARGET_NO_EVICT (-3) when nothing was evicted.
 * assign[P*S] and use_cpu[N*S] are updated in place.  Any row degree (the
 * evicted pod's count table lives in the LDS, or in global work areas when its
 * distinct nodes overflow it).  Scenarios are independent: after a per-call
 * setup (pod lists, hazard flags, per-64-node-block maxima) one launch runs
 * every round, a workgroup per scenario.
 * rsk_rounds_create deduplicates the CSR (self edges dropped, main.py:73) and
 * uploads it with pod_cpu[P] (millicores).                                   */
#define RSK_TARGET_NO_EVICT (-3)
int rsk_rounds_create(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                      const int32_t *pod_cpu, rsk_rounds **out);
int rsk_rounds_destroy(rsk_rounds *r);
int rsk_rounds_run(rsk_rounds *r, int32_t *assign, int32_t S, const int32_t *cap_cpu, int32_t *use_cpu,
                   int32_t N, int32_t threshold, int32_t R, int32_t *out_evict, int32_t *out_target,
                   uint32_t flags);
/* One round's placement step alone (the pod-row-sharded loop, rsk/dist.py
 * RowShardedRounds): out_target[s] = the CAR target of pod evict[s] against
 * assign / use_cpu / hazard (as rsk_rounds_run computes it), no state update;
 * RSK_TARGET_NO_EVICT where evict[s] < 0.                                    */
int rsk_rounds_place(rsk_rounds *r, const int32_t *assign, int32_t S, const int32_t *cap_cpu,
                     const int32_t *use_cpu, const uint8_t *hazard, int32_t N, const int32_t *evict,
                     int32_t *out_target, uint32_t flags);
/* The row-sharded loop's per-round glue, one launch each (device pointers,
 * RSK_F_DEVICE required):
 * rsk_rows_evict_key: this rank's eviction candidates -> the all-reduce MAX
 *   key of delete_replaced_pod.py:47-57's first max (cpu, lowest pod):
 *   key[s] = local_pod[s] >= 0 ? pod_cpu[g] << 32 | (2^32 - 1 - g) : -1 with
 *   g = r0 + local_pod[s];
 * rsk_rows_evict_decode: the reduced key -> evict[s] (global pod in [0, P),
 *   -1 none; a key that decodes outside [0, P) also gives -1);
 * rsk_rows_apply: the move of round r (main.py:73-91's edit + placement, the
 *   build-defined state update): where evict[s] in [0, P) and target[s] in
 *   [0, N), assign[evict*S+s] = target[s]; when the pod is in rows [r0, r1)
 *   (r1 <= P) its CPU / memory move between this rank's per-node partials
 *   cpu_part / mem_part [N*S] (old node only when it was in [0, N)), and
 *   its u16 shadow shadow16[(e-r0)*S+s] (the rank's rows; null: none) takes
 *   the target; any other evict / target leaves the scenario untouched.
 * rsk_rows_cut_delta: before rsk_rows_apply, cut_inout[s] += the change of
 *   the directed cut over rows [r0, r1) (rsk_cut_cost_rows' count,
 *   communicationcost.py:37-45) that the round's move of evict[s] to
 *   target[s] makes: the edges of row e and the rows holding e (rev_ptr /
 *   rev_idx: the CSR's transpose); same move rule as rsk_rows_apply.
 * rsk_pick_max_pod16: rsk_pick_max_pod over a u16 shadow of assign (node ids
 *   < N <= 65535, 0xffff elsewhere; S % 8 == 0, 16-B aligned): half the
 *   bytes of the scan.                                                       */
int rsk_rows_evict_key(rsk_ctx *ctx, const int32_t *local_pod, int32_t S, int32_t r0, const int32_t *pod_cpu,
                       int64_t *out_key, uint32_t flags);
int rsk_rows_evict_decode(rsk_ctx *ctx, const int64_t *key, int32_t S, int32_t P, int32_t *out_evict,
                          uint32_t flags);
int rsk_rows_apply(rsk_ctx *ctx, int32_t *assign, int32_t S, const int32_t *evict, const int32_t *target,
                   int32_t r0, int32_t r1, int32_t P, int32_t N, const int32_t *pod_cpu, const int64_t *pod_mem,
                   int64_t *cpu_part, int64_t *mem_part, uint16_t *shadow16, uint32_t flags);
int rsk_rows_cut_delta(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *rev_ptr,
                       const int32_t *rev_idx, int32_t P, int32_t r0, int32_t r1, const int32_t *assign, int32_t S,
                       const int32_t *evict, const int32_t *target, int32_t N, int64_t *cut_inout, uint32_t flags);
int rsk_pick_max_pod16(rsk_ctx *ctx, const uint16_t *assign16, const int32_t *pod_cpu, int32_t P, int32_t S,
                       const int32_t *most, int32_t *out_pod, uint32_t flags);
/* The row-sharded round fused into four launches (device pointers, RSK_F_DEVICE
 * required).  key_evict [S] is zero before the first round and rsk_rows_place
 * leaves it zero for the next one; key_most / zc_cnt / zc_key [S] come from
 * rsk_rows_detect_setup, and rsk_rows_move rewrites them every round.
 * rsk_rows_pick: delete_replaced_pod.py:41-61 over this rank's q rows (int32
 *   assign rows or the u16 shadow, elem_bytes 4 / 2; pod r0 + p): key_evict[s]
 *   = atomic max of pod_cpu[g] << 32 | (2^32 - 1 - g) over its pods on the
 *   most hazardous node (0: none) -- the MAX all-reduce key.
 * rsk_rows_place: the CAR target (rescheduling.py:174-218) of the reduced key's
 *   pod when it is in rows [r0, r1), else RSK_TARGET_NO_EVICT; out_evict[s] =
 *   the decoded pod (-1 none) on every rank.  The zero case comes from the
 *   detect words rsk_rows_detect_setup / rsk_rows_move keep.
 * rsk_rows_move: rsk_rows_cut_delta then rsk_rows_apply in one launch.  With
 *   blk (rsk_rows_blk_bytes(N, S) bytes of device memory) it also keeps the
 *   round's state in step on every rank (the moves are known to all ranks
 *   after the target all-gather): use_cpu (the usage replica) -= / += the
 *   pod's CPU, the two changed nodes' hazard flags, the per-(scenario,
 *   64-node block) maxima in blk, and key_most / zc_cnt / zc_key for the next
 *   round (rsk_rows_place zeroes them) — no per-round detect pass and no
 *   all-reduce of the usage partials.
 * rsk_rows_detect_setup: the blk state, hazard flags, key_most and the zero
 *   case from a usage array (the loop's round 0).                           */
int rsk_rows_pick(rsk_ctx *ctx, const void *rows, int32_t elem_bytes, int32_t q, int32_t S, int32_t r0,
                  const int32_t *pod_cpu, const int64_t *key_most, int64_t *key_evict, uint32_t flags);
int rsk_rows_place(rsk_rounds *r, const int32_t *assign, int32_t S, const int32_t *cap_cpu, const int32_t *use_cpu,
                   const uint8_t *hazard, int32_t N, int32_t r0, int32_t r1, int64_t *key_most, int64_t *key_evict,
                   int32_t *zc_cnt, int64_t *zc_key, int32_t *out_evict, int32_t *out_target, uint32_t flags);
int rsk_rows_move(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *rev_ptr,
                  const int32_t *rev_idx, int32_t P, int32_t r0, int32_t r1, int32_t *assign, int32_t S,
                  const int32_t *evict, const int32_t *target, int32_t N, const int32_t *pod_cpu, const int64_t *pod_mem,
                  int64_t *cpu_part, int64_t *mem_part, uint16_t *shadow16, int64_t *cut_inout, int32_t *use_cpu,
                  const int32_t *cap_cpu, int32_t threshold, uint8_t *hazard, void *blk, int64_t *key_most,
                  int32_t *zc_cnt, int64_t *zc_key, uint32_t flags);
int64_t rsk_rows_blk_bytes(int32_t N, int32_t S);
int rsk_rows_detect_setup(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S,
                          int32_t threshold, uint8_t *out_hazard, void *blk, int64_t *key_most, int32_t *zc_cnt,
                          int64_t *zc_key, uint32_t flags);

/* ---- µBench workmodel -> relation CSR (host only, no device) -----------------
 * The caller's on-disk format (workmodelC.json).  One
 * streaming pass over the JSON (mmap for _load): every service key and every
 * name under external_services[*].services is interned, nothing else is
 * materialised.  The relation is the one the reference hard-codes
 * (main.py:31-52, communicationcost.py:69-88): rel(s) = callees(s) ∪
 * callers(s), self calls dropped, deduplicated, columns ascending.  Rows are
 * the defined services in file order, then callees never defined, in order of
 * first mention (json.load's dict order; rsk/workmodel.py restates it).
 * _names writes the P names NUL-separated (name_bytes from _sizes).          */
typedef struct rsk_workmodel rsk_workmodel;
int rsk_workmodel_parse(const char *json, int64_t len, rsk_workmodel **out);
int rsk_workmodel_load(const char *path, rsk_workmodel **out);
int rsk_workmodel_sizes(const rsk_workmodel *wm, int32_t *P, int64_t *nnz, int64_t *name_bytes);
int rsk_workmodel_csr(const rsk_workmodel *wm, int32_t *row_ptr, int32_t *col_idx);
int rsk_workmodel_names(const rsk_workmodel *wm, char *buf);
int rsk_workmodel_destroy(rsk_workmodel *wm);

/* ---- Kubernetes quantity strings -> integers (host only, no device) --------
 * The snapshot replay of cluster_monitoring.  Replaces the
 * per-value calls of unit_convertion.py:1-32 (cpu_conversion -> millicores,
 * mem_conversion -> bytes) made by get_resource_usage.py:11-12,33-34,63-64.
 * Element i is buf[offs[i] .. offs[i+1]) (n+1 offsets).  status[i] = 0: out[i]
 * holds the reference's value; 1: outside the plain decimal grammar or int64
 * (underscores, inf/nan, non-ASCII, malformed) -- the caller converts it with
 * the Python restatement (rsk/snapshot.py), which also raises the reference's
 * exception for malformed text.                                              */
#define RSK_QTY_CPU 0
#define RSK_QTY_MEM 1
int rsk_parse_quantities(const char *buf, const int64_t *offs, int64_t n, int32_t kind, int64_t *out,
                         uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif /* RSK_H */
