/*
 * rsk_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-purpose restatement of the reference's placement-scoring
 * algorithms (ye0nj00/Kubernetes-Rescheduling) on the flat batched layouts of
 * include/rsk.h.  It is the CHECKER for the HIP path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product library (librsk.so) never links or calls it.
 *
 * Pinned against the reference: tests/test_oracle_golden.py checks every
 * function here against the golden fixtures in tests/golden/, which
 * tests/golden/make_golden.py produced by running the reference's own Python
 * (through a stub `kubernetes` client) in the build container.
 *
 * Layouts (scenario-minor, as in include/rsk.h):
 *   assign[p*S + s]  node index of pod p in scenario s (-1 = not scheduled)
 *   use_cpu[n*S + s], hazard[n*S + s], cpu_pct[n*S + s], pod_count[n*S + s]
 *   cap_cpu[n], name_rank[n] (rank of node n's name in Python str order)
 * Target codes: >=0 node index, -1 = None, -2 = no candidate (reference raises).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TGT_NONE (-1)
#define TGT_NO_CANDIDATE (-2)

/* ------------------------------------------------------------------------
 * CAR — rescheduling.py:174-218 (`communication`), pod-level batched form.
 *
 * For row p and scenario s the reference, after edit_cluster removed p from
 * the cluster (main.py:73, main.py:10-19), does:
 *   for n in nodes_name (index order), skipping hazard nodes      (:188-190)
 *     score[n] = #pods q on n with dep(q) in rel(dep(p))          (:192-195)
 *   max_score = max(score.values())  -> ValueError if empty        (:199)
 *   best = [n with score == max], in nodes_name order              (:200)
 *   if len(best) > 1: first n with the largest cap-use, starting
 *      from max_remaining = -1 with a strict '>' -> None if none    (:202-212)
 *   else best[0]                                                   (:213-214)
 * Here rel(dep(p)) is CSR row p; q == p is skipped (the evicted pod).
 * ---------------------------------------------------------------------- */
static void car_one(const int32_t *row_ptr, const int32_t *col_idx, int32_t p,
                    const int32_t *assign, int32_t S, int32_t s,
                    const int32_t *cap, const int32_t *use, const uint8_t *hazard,
                    int32_t N, int32_t *score, int32_t *target, int32_t *max_out)
{
    for (int32_t n = 0; n < N; ++n) score[n] = hazard[(int64_t)n * S + s] ? -1 : 0;
    for (int32_t k = row_ptr[p]; k < row_ptr[p + 1]; ++k) {
        int32_t q = col_idx[k];
        if (q == p) continue;
        int32_t a = assign[(int64_t)q * S + s];
        if (a < 0 || a >= N) continue;
        if (score[a] >= 0) score[a] += 1;
    }
    int32_t m = -1;
    for (int32_t n = 0; n < N; ++n)
        if (score[n] >= 0 && score[n] > m) m = score[n];
    if (m < 0) { *target = TGT_NO_CANDIDATE; *max_out = -1; return; }
    int32_t nbest = 0, first = -1;
    for (int32_t n = 0; n < N; ++n)
        if (score[n] == m) { if (first < 0) first = n; ++nbest; }
    *max_out = m;
    if (nbest == 1) { *target = first; return; }
    int64_t rmax = -1;
    int32_t t = TGT_NONE;
    for (int32_t n = 0; n < N; ++n) {
        if (score[n] != m) continue;
        int64_t rem = (int64_t)cap[n] - (int64_t)use[(int64_t)n * S + s];
        if (rem > rmax) { rmax = rem; t = n; }
    }
    *target = t;
}

int oracle_car(const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
               const int32_t *assign, int32_t S, const int32_t *cap,
               const int32_t *use, const uint8_t *hazard, int32_t N,
               const int32_t *rows, int32_t Q, int32_t *out_target,
               int32_t *out_score, int nthreads)
{
    if (!rows) Q = P;
    int any_nc = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(|| : any_nc)
#endif
    {
        int32_t *score = (int32_t *)malloc(sizeof(int32_t) * (N > 0 ? N : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int64_t i = 0; i < (int64_t)Q; ++i) {
            int32_t p = rows ? rows[i] : (int32_t)i;
            for (int32_t s = 0; s < S; ++s) {
                int32_t t, m;
                car_one(row_ptr, col_idx, p, assign, S, s, cap, use, hazard, N, score, &t, &m);
                out_target[i * S + s] = t;
                if (out_score) out_score[i * S + s] = m;
                if (t == TGT_NO_CANDIDATE) any_nc = 1;
            }
        }
        free(score);
    }
    (void)nthreads;
    return any_nc ? 1 : 0;
}

/* ------------------------------------------------------------------------
 * CAR, sparse restatement — the same decision as car_one (rescheduling.py:
 * 188-214) without the O(N) passes per cell, so every cell of a full-size
 * batch can be checked (tests/test_gpu_headline.py).  Every non-hazard node
 * the row does not reach scores 0, so:
 *   - no neighbour lands on a non-hazard node -> max score 0 (or no candidate):
 *     every non-hazard node ties, a per-scenario constant ("zero case")
 *     computed once per scenario by car_one's own tie rule;
 *   - otherwise the maximum is >= 1 and only reached nodes can hold it: count
 *     the row's entries per node (duplicates count, as in car_one), take the
 *     nodes at the maximum, a single one wins outright, else the first in index
 *     order with the largest rem > -1 (None when every rem <= -1).
 * Pinned to car_one (oracle_car) on random graphs and to the golden fixtures
 * in tests/test_oracle_golden.py.  Work is split over (16-scenario block, row
 * chunk) items so one block's hazard / use bytes stay in the core's cache.
 * ---------------------------------------------------------------------- */
int oracle_car_sparse(const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                      const int32_t *assign, int32_t S, const int32_t *cap,
                      const int32_t *use, const uint8_t *hazard, int32_t N,
                      const int32_t *rows, int32_t Q, int32_t *out_target,
                      int32_t *out_score, int nthreads)
{
    if (!rows) Q = P;
    int32_t *zt = (int32_t *)malloc(sizeof(int32_t) * (S > 0 ? S : 1));
    int32_t *zm = (int32_t *)malloc(sizeof(int32_t) * (S > 0 ? S : 1));
    int32_t maxdeg = 1;
    for (int64_t i = 0; i < (int64_t)Q; ++i) {
        int32_t p = rows ? rows[i] : (int32_t)i;
        int32_t d = row_ptr[p + 1] - row_ptr[p];
        if (d > maxdeg) maxdeg = d;
    }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int32_t s = 0; s < S; ++s) {  /* the zero case: car_one with an empty row */
        int32_t nc = 0, first = -1, t = TGT_NONE;
        int64_t rmax = -1;
        for (int32_t n = 0; n < N; ++n) {
            if (hazard[(int64_t)n * S + s]) continue;
            if (first < 0) first = n;
            ++nc;
            int64_t rem = (int64_t)cap[n] - (int64_t)use[(int64_t)n * S + s];
            if (rem > rmax) { rmax = rem; t = n; }
        }
        zt[s] = nc == 0 ? TGT_NO_CANDIDATE : (nc == 1 ? first : t);
        zm[s] = nc == 0 ? -1 : 0;
    }
    const int32_t SB = 16, RC = 2048;
    const int64_t nblk = ((int64_t)S + SB - 1) / SB, nrc = ((int64_t)Q + RC - 1) / RC;
    int any_nc = 0;
#ifdef _OPENMP
#pragma omp parallel reduction(|| : any_nc)
#endif
    {
        int32_t *cnt = (int32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
        int32_t *touched = (int32_t *)malloc(sizeof(int32_t) * (size_t)maxdeg);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t item = 0; item < nblk * nrc; ++item) {
            const int32_t s0 = (int32_t)(item / nrc) * SB;
            const int32_t s1 = s0 + SB < S ? s0 + SB : S;
            const int64_t i0 = (item % nrc) * RC, i1 = i0 + RC < Q ? i0 + RC : Q;
            for (int64_t i = i0; i < i1; ++i) {
                const int32_t p = rows ? rows[i] : (int32_t)i;
                for (int32_t s = s0; s < s1; ++s) {
                    int32_t nt = 0;
                    for (int32_t k = row_ptr[p]; k < row_ptr[p + 1]; ++k) {
                        const int32_t q = col_idx[k];
                        if (q == p) continue;
                        const int32_t a = assign[(int64_t)q * S + s];
                        if (a < 0 || a >= N || hazard[(int64_t)a * S + s]) continue;
                        if (cnt[a]++ == 0) touched[nt++] = a;
                    }
                    int32_t t, m = 0;
                    if (nt == 0) {
                        t = zt[s];
                        m = zm[s];
                    } else {
                        int32_t nbest = 0, only = -1;
                        for (int32_t j = 0; j < nt; ++j) {
                            const int32_t c = cnt[touched[j]];
                            if (c > m) { m = c; nbest = 1; only = touched[j]; }
                            else if (c == m) ++nbest;
                        }
                        if (nbest == 1) {
                            t = only;
                        } else {
                            int64_t rmax = -1;
                            t = TGT_NONE;
                            for (int32_t j = 0; j < nt; ++j) {
                                const int32_t n = touched[j];
                                if (cnt[n] != m) continue;
                                const int64_t rem = (int64_t)cap[n] - (int64_t)use[(int64_t)n * S + s];
                                if (rem > rmax || (rem == rmax && t >= 0 && n < t)) { rmax = rem; t = n; }
                            }
                        }
                        for (int32_t j = 0; j < nt; ++j) cnt[touched[j]] = 0;
                    }
                    out_target[i * S + s] = t;
                    if (out_score) out_score[i * S + s] = m;
                    if (t == TGT_NO_CANDIDATE) any_nc = 1;
                }
            }
        }
        free(touched);
        free(cnt);
    }
    free(zt);
    free(zm);
    (void)nthreads;
    return any_nc ? 1 : 0;
}

/* ------------------------------------------------------------------------
 * spread — rescheduling.py:89-101: min over non-hazard nodes of
 * (len(pods), nodename); ties -> smallest name in str order.  RuntimeError if
 * none (:98-99).  binpack — rescheduling.py:121-133: max of (cpu_pct, name).
 * ---------------------------------------------------------------------- */
void oracle_spread(const int32_t *pod_count, const int32_t *name_rank, const uint8_t *hazard,
                   int32_t N, int32_t S, int32_t *out_node)
{
    for (int32_t s = 0; s < S; ++s) {
        int32_t best = TGT_NO_CANDIDATE;
        for (int32_t n = 0; n < N; ++n) {
            if (hazard[(int64_t)n * S + s]) continue;
            if (best < 0) { best = n; continue; }
            int32_t c = pod_count[(int64_t)n * S + s], cb = pod_count[(int64_t)best * S + s];
            if (c < cb || (c == cb && name_rank[n] < name_rank[best])) best = n;
        }
        out_node[s] = best;
    }
}

void oracle_binpack(const int32_t *cpu_pct, const int32_t *name_rank, const uint8_t *hazard,
                    int32_t N, int32_t S, int32_t *out_node)
{
    for (int32_t s = 0; s < S; ++s) {
        int32_t best = TGT_NO_CANDIDATE;
        for (int32_t n = 0; n < N; ++n) {
            if (hazard[(int64_t)n * S + s]) continue;
            if (best < 0) { best = n; continue; }
            int32_t c = cpu_pct[(int64_t)n * S + s], cb = cpu_pct[(int64_t)best * S + s];
            if (c > cb || (c == cb && name_rank[n] > name_rank[best])) best = n;
        }
        out_node[s] = best;
    }
}

/* ------------------------------------------------------------------------
 * random — rescheduling.py:149-153: candidates = [n for n in nodes_name if n
 * not in hazard]; rd.choice(candidates) = candidates[_randbelow(len)].
 * CPython's Random: MT19937 seeded by init_by_array(abs(seed) as 32-bit
 * little-endian words, [0] for 0); _randbelow_with_getrandbits(n):
 * k = n.bit_length(); r = getrandbits(k) while r >= n;
 * getrandbits(k <= 32) = genrand_uint32() >> (32 - k).
 * ---------------------------------------------------------------------- */
typedef struct { uint32_t mt[624]; int idx; } mt_state;

static void mt_init_genrand(mt_state *st, uint32_t s)
{
    st->mt[0] = s;
    for (int i = 1; i < 624; ++i)
        st->mt[i] = 1812433253u * (st->mt[i - 1] ^ (st->mt[i - 1] >> 30)) + (uint32_t)i;
    st->idx = 624;
}

static void mt_init_by_array(mt_state *st, const uint32_t *key, int len)
{
    mt_init_genrand(st, 19650218u);
    int i = 1, j = 0;
    int k = 624 > len ? 624 : len;
    for (; k; --k) {
        st->mt[i] = (st->mt[i] ^ ((st->mt[i - 1] ^ (st->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        ++i; ++j;
        if (i >= 624) { st->mt[0] = st->mt[623]; i = 1; }
        if (j >= len) j = 0;
    }
    for (k = 623; k; --k) {
        st->mt[i] = (st->mt[i] ^ ((st->mt[i - 1] ^ (st->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        ++i;
        if (i >= 624) { st->mt[0] = st->mt[623]; i = 1; }
    }
    st->mt[0] = 0x80000000u;
    st->idx = 624;
}

static uint32_t mt_next(mt_state *st)
{
    if (st->idx >= 624) {
        for (int kk = 0; kk < 624; ++kk) {
            uint32_t y = (st->mt[kk] & 0x80000000u) | (st->mt[(kk + 1) % 624] & 0x7fffffffu);
            st->mt[kk] = st->mt[(kk + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        st->idx = 0;
    }
    uint32_t y = st->mt[st->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* Python `random.Random(seed)._randbelow(n)` for 0 < n < 2^31, seed >= 0. */
int32_t oracle_py_randbelow(uint64_t seed, int32_t n)
{
    mt_state st;
    uint32_t key[2];
    int len = 0;
    if (seed == 0) { key[0] = 0; len = 1; }
    else { key[len++] = (uint32_t)seed; if (seed >> 32) key[len++] = (uint32_t)(seed >> 32); }
    mt_init_by_array(&st, key, len);
    int k = 0;
    while (k < 32 && ((uint32_t)n >> k)) ++k;
    uint32_t r;
    do { r = mt_next(&st) >> (32 - k); } while (r >= (uint32_t)n);
    return (int32_t)r;
}

void oracle_random(const uint8_t *hazard, int32_t N, int32_t S, const uint64_t *seeds,
                   int32_t *out_node, int32_t *out_count)
{
    for (int32_t s = 0; s < S; ++s) {
        int32_t cnt = 0;
        for (int32_t n = 0; n < N; ++n) cnt += !hazard[(int64_t)n * S + s];
        if (out_count) out_count[s] = cnt;
        if (cnt == 0) { out_node[s] = TGT_NO_CANDIDATE; continue; }
        int32_t r = oracle_py_randbelow(seeds[s], cnt);
        int32_t t = TGT_NO_CANDIDATE;
        for (int32_t n = 0; n < N; ++n)
            if (!hazard[(int64_t)n * S + s]) { if (r == 0) { t = n; break; } --r; }
        out_node[s] = t;
    }
}

/* ------------------------------------------------------------------------
 * cpu_pct — get_resource_usage.py:37: int(round(u / c * 100)), -1 if c == 0.
 * fp64 divide, then multiply, then round-half-even (this file is compiled
 * with -ffp-contract=off so nothing fuses).
 * detection — harzard_detect.py:3-27: hazard = pct >= threshold (:12); most =
 * first max pct among hazard nodes in node order (:24, dict max first-wins);
 * -1 (the reference's '') if none.
 * ---------------------------------------------------------------------- */
void oracle_cpu_pct(const int32_t *use, const int32_t *cap, int32_t N, int32_t S, int32_t *out_pct)
{
    for (int64_t n = 0; n < N; ++n)
        for (int64_t s = 0; s < S; ++s) {
            int64_t i = n * S + s;
            if (cap[n] == 0) { out_pct[i] = -1; continue; }
            volatile double q = (double)use[i] / (double)cap[n];
            volatile double x = q * 100.0;
            out_pct[i] = (int32_t)rint(x);
        }
}

void oracle_detect(const int32_t *cpu_pct, int32_t N, int32_t S, int32_t threshold,
                   uint8_t *out_hazard, int32_t *out_most)
{
    for (int32_t s = 0; s < S; ++s) {
        int32_t most = -1, mp = 0;
        for (int32_t n = 0; n < N; ++n) {
            int32_t v = cpu_pct[(int64_t)n * S + s];
            int h = v >= threshold;
            out_hazard[(int64_t)n * S + s] = (uint8_t)h;
            if (h && (most < 0 || v > mp)) { most = n; mp = v; }
        }
        out_most[s] = most;
    }
}

/* pick_max_pod — delete_replaced_pod.py:41-61: over pods in list order on
 * node `most`, strict '>' on cpu starting from -1 -> first max; -1 if none. */
void oracle_pick_max_pod(const int32_t *assign, const int32_t *pod_cpu, int32_t P, int32_t S,
                         const int32_t *most, int32_t *out_pod)
{
    for (int32_t s = 0; s < S; ++s) {
        int32_t best = -1;
        int64_t bc = -1;
        for (int32_t p = 0; p < P; ++p) {
            if (most[s] < 0 || assign[(int64_t)p * S + s] != most[s]) continue;
            if ((int64_t)pod_cpu[p] > bc) { bc = pod_cpu[p]; best = p; }
        }
        out_pod[s] = best;
    }
}

/* ------------------------------------------------------------------------
 * Node reductions (kernel 3 semantics).
 * node_reduce: per (node, scenario) pod count and CPU / memory sums.
 * load_std — nodemonitor.py:24-46: pct_n = use_n / cap_n * 100 in fp64 (not
 *   rounded), nodes with cap <= 0 skipped (:38-43), numpy.std (population,
 *   ddof=0) of the list; 0.0 if empty (:47-50).  Two-pass mean / variance.
 * cut_cost — communicationcost.py:37-45: for each row p, each related q:
 *   count [node(p) != node(q)] where an unscheduled pod (-1) or a missing
 *   deployment (missing[p] extra relations) reads as None and None == None.
 *   Returns the DIRECTED count; the reference reports it / 2 as a float.
 * ---------------------------------------------------------------------- */
void oracle_node_reduce(const int32_t *assign, int32_t P, int32_t S, const int32_t *pod_cpu,
                        const int64_t *pod_mem, int32_t N, int32_t *pod_count,
                        int64_t *cpu_sum, int64_t *mem_sum)
{
    memset(pod_count, 0, sizeof(int32_t) * (size_t)N * S);
    memset(cpu_sum, 0, sizeof(int64_t) * (size_t)N * S);
    if (mem_sum) memset(mem_sum, 0, sizeof(int64_t) * (size_t)N * S);
    for (int64_t p = 0; p < P; ++p)
        for (int64_t s = 0; s < S; ++s) {
            int32_t a = assign[p * S + s];
            if (a < 0 || a >= N) continue;
            pod_count[(int64_t)a * S + s] += 1;
            cpu_sum[(int64_t)a * S + s] += pod_cpu[p];
            if (mem_sum) mem_sum[(int64_t)a * S + s] += pod_mem[p];
        }
}

void oracle_load_std(const int32_t *use, const int32_t *cap, int32_t N, int32_t S, double *out_std)
{
    for (int32_t s = 0; s < S; ++s) {
        double sum = 0.0;
        int64_t cnt = 0;
        for (int32_t n = 0; n < N; ++n) {
            if (cap[n] <= 0) continue;
            sum += (double)use[(int64_t)n * S + s] / (double)cap[n] * 100.0;
            ++cnt;
        }
        if (!cnt) { out_std[s] = 0.0; continue; }
        double mean = sum / (double)cnt, ss = 0.0;
        for (int32_t n = 0; n < N; ++n) {
            if (cap[n] <= 0) continue;
            double d = (double)use[(int64_t)n * S + s] / (double)cap[n] * 100.0 - mean;
            ss += d * d;
        }
        out_std[s] = sqrt(ss / (double)cnt);
    }
}

void oracle_cut_cost(const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                     const int32_t *assign, int32_t S, const int32_t *missing, int64_t *out_directed)
{
    /* the same integer count per scenario, walked row-major so the scenario
     * words of a row are contiguous (an exact sum: the order does not matter) */
    memset(out_directed, 0, sizeof(int64_t) * (size_t)S);
    for (int32_t p = 0; p < P; ++p) {
        const int32_t *ap = assign + (int64_t)p * S;
        for (int32_t k = row_ptr[p]; k < row_ptr[p + 1]; ++k) {
            const int32_t *bq = assign + (int64_t)col_idx[k] * S;
            for (int32_t s = 0; s < S; ++s) out_directed[s] += (ap[s] != bq[s]);
        }
        if (missing && missing[p])
            for (int32_t s = 0; s < S; ++s) out_directed[s] += (ap[s] != -1) ? missing[p] : 0;
    }
}

/* ------------------------------------------------------------------------
 * rounds — the control loop of main.py:55-110 for S independent scenarios,
 * R rounds, with the build-defined state update of SURVEY.md §8f item 1 (the
 * reference re-measures the live cluster each round instead):
 *   pct = cpu_pct(use, cap)                     get_resource_usage.py:37
 *   hazard, most = detection(pct >= threshold)  harzard_detect.py:3-27
 *   if most: p = pick_max_pod(most)             delete_replaced_pod.py:41-61
 *     if p: t = communication(p)                rescheduling.py:174-218
 *           (p off the cluster, main.py:73: its own entry never counts)
 *           t >= 0: use[old] -= cpu[p]; use[t] += cpu[p]; assign[p] = t
 * out_evict[r*S+s] = p (-1 none); out_target[r*S+s] = t, or -3 when nothing
 * was evicted.  Expects a deduplicated CSR (car_one counts every entry).
 * ---------------------------------------------------------------------- */
void oracle_rounds(const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *pod_cpu,
                   int32_t *assign, int32_t S, const int32_t *cap, int32_t *use, int32_t N,
                   int32_t threshold, int32_t R, int32_t *out_evict, int32_t *out_target)
{
    int32_t *pct = (int32_t *)malloc(sizeof(int32_t) * (size_t)N * S);
    uint8_t *haz = (uint8_t *)malloc((size_t)N * S);
    int32_t *most = (int32_t *)malloc(sizeof(int32_t) * (size_t)S);
    int32_t *score = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    for (int32_t r = 0; r < R; ++r) {
        int32_t *ev = out_evict + (int64_t)r * S, *tg = out_target + (int64_t)r * S;
        oracle_cpu_pct(use, cap, N, S, pct);
        oracle_detect(pct, N, S, threshold, haz, most);
        oracle_pick_max_pod(assign, pod_cpu, P, S, most, ev);
        for (int32_t s = 0; s < S; ++s) {
            int32_t p = ev[s], t, m;
            if (p < 0) { tg[s] = -3; continue; }
            car_one(row_ptr, col_idx, p, assign, S, s, cap, use, haz, N, score, &t, &m);
            tg[s] = t;
            if (t >= 0) {
                int32_t old = assign[(int64_t)p * S + s];
                if (old >= 0 && old < N) use[(int64_t)old * S + s] -= pod_cpu[p];
                use[(int64_t)t * S + s] += pod_cpu[p];
                assign[(int64_t)p * S + s] = t;
            }
        }
    }
    free(pct);
    free(haz);
    free(most);
    free(score);
}

/* oracle_rounds over the S scenarios in parallel.  Scenarios never share
 * state in main.py's loop as restated above (each one's assign / use column,
 * hazard flags and most-hazardous node are its own), so scenario s is the
 * S = 1 run of oracle_rounds on its own contiguous columns: gathered, run,
 * scattered back.  Same results as oracle_rounds (tests/test_rounds.py pins
 * the two to each other); a thread per scenario at a time. */
void oracle_rounds_par(const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *pod_cpu,
                       int32_t *assign, int32_t S, const int32_t *cap, int32_t *use, int32_t N,
                       int32_t threshold, int32_t R, int32_t *out_evict, int32_t *out_target, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)(P > 0 ? P : 1));
        int32_t *u = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
        int32_t *ev = (int32_t *)malloc(sizeof(int32_t) * (size_t)(R > 0 ? R : 1));
        int32_t *tg = (int32_t *)malloc(sizeof(int32_t) * (size_t)(R > 0 ? R : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int32_t s = 0; s < S; ++s) {
            for (int64_t p = 0; p < P; ++p) a[p] = assign[p * S + s];
            for (int64_t n = 0; n < N; ++n) u[n] = use[n * S + s];
            oracle_rounds(row_ptr, col_idx, P, pod_cpu, a, 1, cap, u, N, threshold, R, ev, tg);
            for (int64_t p = 0; p < P; ++p) assign[p * S + s] = a[p];
            for (int64_t n = 0; n < N; ++n) use[n * S + s] = u[n];
            for (int64_t r = 0; r < R; ++r) {
                out_evict[r * S + s] = ev[r];
                out_target[r * S + s] = tg[r];
            }
        }
        free(a);
        free(u);
        free(ev);
        free(tg);
    }
    (void)nthreads;
}
