/*
 * san_core.c -- TEST INFRASTRUCTURE ONLY: the core API subset the drop-in host C
 * (hsa_amd/csrc/bwtaln_gpu.c, bwtgap_gpu.c) calls, answered by the CPU restatement
 * (oracle/hsa_oracle.c) instead of the GPU, so that the host C can be built and run
 * under AddressSanitizer / UndefinedBehaviorSanitizer on a machine without a GPU
 * (tests/test_sanitize.py).  The product library never contains this file.
 *
 * Semantics follow include/hsa_gpu.h: hsa_search_batch = per job, bwt_cal_width of
 * the seed and the read, bwt_match_gap on the rc strand then the forward strand
 * (bwtaln.c:337-373); hsa_match_gap_batch = bwt_match_gap with the caller's widths;
 * hsa_width_batch = bwt_cal_width.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hsa_gpu.h"
#include "../../oracle/hsa_oracle.h"

static char g_err[256] = "";

const char *hsa_last_error(void) { return g_err; }
void hsa_gpu_set_error_text(const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); }
int hsa_device_count(void) { return 1; }
void hsa_free(void *p) { free(p); }

int hsa_index_create(int device, uint32_t T, uint32_t isa0, const uint32_t C[5], const uint32_t *code, uint32_t rT,
                     uint32_t risa0, const uint32_t rC[5], const uint32_t *rcode, hsa_index_t **out)
{
    (void)device;
    *out = (hsa_index_t *)or_index_create(T, isa0, C, code, rT, risa0, rC, rcode);
    return *out ? 0 : HSA_E_MEM;
}

/* hsa_index_clone: the same restatement index under a reference count (a clone shares
 * everything here; the drop-in makes one for a second slot on a device) */
static struct { hsa_index_t *ix; int refs; } g_refs[32];

int hsa_index_clone(hsa_index_t *src, hsa_index_t **out)
{
    for (int i = 0; i < 32; ++i)
        if (g_refs[i].ix == src) { ++g_refs[i].refs; *out = src; return 0; }
    for (int i = 0; i < 32; ++i)
        if (!g_refs[i].ix) { g_refs[i].ix = src; g_refs[i].refs = 2; *out = src; return 0; }
    return HSA_E_MEM;
}

void hsa_index_free(hsa_index_t *ix)
{
    for (int i = 0; i < 32; ++i)
        if (g_refs[i].ix == ix) {
            if (--g_refs[i].refs > 0) return;
            g_refs[i].ix = NULL;
            break;
        }
    or_index_free((or_index_t *)ix);
}

/* the sampled SA and chromosome blocks of the (one) attached index */
static uint32_t *g_sa_vals, *g_sa_blocks, g_sa_interval;
static int g_sa_nblocks;

/* the unique-interval walk changes no result: the CPU stand-in has nothing to build */
int hsa_index_build_walk(hsa_index_t *ix, const uint32_t *d_sa_full, const uint32_t *d_text_lsb)
{
    (void)ix; (void)d_sa_full; (void)d_text_lsb;
    return 0;
}

int hsa_index_set_sa(hsa_index_t *ix, const uint32_t *sa, uint64_t n, uint32_t interval, const uint32_t *blocks,
                     int n_blocks)
{
    (void)ix;
    free(g_sa_vals); free(g_sa_blocks);
    g_sa_vals = (uint32_t *)malloc(n * 4);
    memcpy(g_sa_vals, sa, n * 4);
    g_sa_blocks = (uint32_t *)malloc((size_t)(n_blocks ? n_blocks : 1) * 16);
    if (n_blocks) memcpy(g_sa_blocks, blocks, (size_t)n_blocks * 16);
    g_sa_interval = interval;
    g_sa_nblocks = n_blocks;
    return 0;
}

/* hsa_sa_position_batch = BWTSaValue + BWTRetrievePositionFromSAIndex (or_sa_position):
 * (occ, seq id, 1-based position, occ), id / position 0xFFFFFFFF when no block holds it. */
int hsa_sa_position_batch(hsa_index_t *ix, size_t n, const uint32_t *sa_index, uint32_t *out4)
{
    if (!g_sa_vals) { hsa_gpu_set_error_text("no suffix array attached"); return HSA_E_ARG; }
    for (size_t i = 0; i < n; ++i) {
        uint32_t sid = 0xFFFFFFFFu, ori = 0xFFFFFFFFu, occ = 0;
        or_sa_position((const or_index_t *)ix, g_sa_vals, g_sa_interval, g_sa_blocks, g_sa_nblocks, sa_index[i], &sid,
                       &ori, &occ);
        out4[4 * i] = occ; out4[4 * i + 1] = sid; out4[4 * i + 2] = ori; out4[4 * i + 3] = occ;
    }
    return 0;
}

static or_opt_t opt_of(const hsa_regime_t *R, const hsa_job_t *J)
{
    or_opt_t o;
    or_init_opt(&o);
    o.s_mm = R->s_mm; o.s_gapo = R->s_gapo; o.s_gape = R->s_gape; o.mode = R->mode;
    o.indel_end_skip = R->indel_end_skip; o.max_del_occ = R->max_del_occ; o.max_entries = R->max_entries;
    o.max_gapo = R->max_gapo; o.max_gape = R->max_gape; o.max_seed_diff = R->max_seed_diff;
    o.max_top2 = R->max_top2;
    o.max_diff = J->max_diff;
    o.seed_len = J->seed_len;
    return o;
}

typedef struct { uint32_t *h; size_t n, cap; } hv_t;

static void hv_add(hv_t *v, const uint32_t *h, int n)
{
    if (v->n + (size_t)n > v->cap) {
        v->cap = (v->n + (size_t)n) * 2 + 16;
        v->h = (uint32_t *)realloc(v->h, v->cap * 9 * sizeof(uint32_t));
    }
    memcpy(v->h + v->n * 9, h, (size_t)n * 9 * sizeof(uint32_t));
    v->n += (size_t)n;
}

long hsa_search_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs, int n_jobs,
                      const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                      uint32_t **hits, hsa_stats_t *stats)
{
    (void)n_regimes; (void)codes_len;
    const or_index_t *ox = (const or_index_t *)ix;
    hv_t all = {NULL, 0, 0};
    if (stats) memset(stats, 0, sizeof *stats);
    for (int j = 0; j < n_jobs; ++j) {
        const hsa_job_t *J = jobs + j;
        const hsa_regime_t *R = regimes + J->regime;
        or_opt_t o = opt_of(R, J);
        const int len = (int)J->len;
        const uint8_t *seq = codes + J->off;
        uint8_t *rc = (uint8_t *)malloc((size_t)len + 1);
        for (int i = 0; i < len; ++i) { const uint8_t c = seq[len - 1 - i]; rc[i] = c < 4 ? (uint8_t)(3 - c) : c; }
        uint32_t *wb = (uint32_t *)calloc(2 * ((size_t)len + 1), sizeof(uint32_t));
        uint32_t *ws = (uint32_t *)calloc(2 * ((size_t)len + 1), sizeof(uint32_t));
        n_aln[j] = 0; flags[j] = HSA_F_FALLBACK; hit_off[j] = all.n;
        for (int s = 1; s >= 0; --s) {                         /* rc strand first (bwtaln.c:343) */
            const uint8_t *sq = s ? rc : seq;
            const int has_seed = len > J->seed_len;
            if (has_seed) or_cal_width(ox, J->seed_len, sq + (len - J->seed_len), ws);
            or_cal_width(ox, len, sq, wb);
            uint32_t *h = NULL;
            const int n = or_match_gap(ox, &o, R->n_stacks, sq, len, s, wb, has_seed ? 1 : 0, ws, &h);
            if (n > 0) {
                h[6] = 0; h[7] = (uint32_t)(len - 1);           /* bwtaln.c:371-372 */
                hv_add(&all, h, n);
                n_aln[j] = n; flags[j] = 0;
                or_free(h);
                break;
            }
            or_free(h);
        }
        free(rc); free(wb); free(ws);
    }
    *hits = all.h ? all.h : (uint32_t *)calloc(9, sizeof(uint32_t));
    return (long)all.n;
}

long hsa_match_gap_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                         const hsa_mg_job_t *mg, int n_jobs, const uint8_t *codes, size_t codes_len,
                         const int32_t *widths, size_t width_pairs, int32_t *widths_out, int32_t *n_aln,
                         uint64_t *hit_off, uint32_t **hits, hsa_stats_t *stats)
{
    (void)n_regimes; (void)codes_len;
    const or_index_t *ox = (const or_index_t *)ix;
    hv_t all = {NULL, 0, 0};
    if (stats) memset(stats, 0, sizeof *stats);
    if (widths_out != widths) memcpy(widths_out, widths, width_pairs * 8);
    for (int j = 0; j < n_jobs; ++j) {
        const hsa_job_t *J = jobs + j;
        const hsa_mg_job_t *M = mg + j;
        or_opt_t o = opt_of(regimes + J->regime, J);
        const int len = (int)J->len;
        uint32_t *wb = (uint32_t *)malloc(8 * ((size_t)len + 1));
        memcpy(wb, widths + 2 * M->wb_off, 8 * ((size_t)len + 1));
        uint32_t *ws = NULL;
        if (M->seed == HSA_SEED_OWN) {
            ws = (uint32_t *)malloc(8 * ((size_t)J->seed_len + 1));
            memcpy(ws, widths + 2 * M->ws_off, 8 * ((size_t)J->seed_len + 1));
        }
        uint32_t *h = NULL;
        const int n = or_match_gap(ox, &o, regimes[J->regime].n_stacks, codes + J->off, len, M->strand, wb,
                                   M->seed == HSA_SEED_OWN ? 1 : M->seed == HSA_SEED_ALIAS ? 2 : 0, ws, &h);
        n_aln[j] = n; hit_off[j] = all.n;
        if (n > 0) hv_add(&all, h, n);
        memcpy(widths_out + 2 * M->wb_off, wb, 8 * ((size_t)len + 1));
        or_free(h); free(wb); free(ws);
    }
    *hits = all.h ? all.h : (uint32_t *)calloc(9, sizeof(uint32_t));
    return (long)all.n;
}

int hsa_width_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens, const uint8_t *codes,
                    size_t codes_len, uint32_t *width_out)
{
    (void)codes_len;
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        or_cal_width((const or_index_t *)ix, (int)lens[i], codes + offs[i], width_out + o);
        o += 2 * ((size_t)lens[i] + 1);
    }
    return 0;
}

/* hsa_extend_batch = bwt_extend_backward / bwt_extend_foreward per call (or_extend). */
int hsa_extend_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs, int n,
                     const uint8_t *codes, const int32_t *bids, size_t win_len, int32_t *ret, int32_t *max_pos,
                     uint32_t *aln_out)
{
    (void)n_regimes; (void)win_len;
    for (int j = 0; j < n; ++j) {
        const hsa_ext_job_t *J = jobs + j;
        const hsa_regime_t *R = regimes + J->regime;
        or_opt_t o;
        or_init_opt(&o);
        o.s_mm = R->s_mm; o.s_gapo = R->s_gapo; o.s_gape = R->s_gape; o.mode = R->mode;
        o.indel_end_skip = R->indel_end_skip; o.max_del_occ = R->max_del_occ; o.max_entries = R->max_entries;
        o.max_gapo = R->max_gapo; o.max_gape = R->max_gape; o.max_diff = R->max_diff;
        memcpy(aln_out + 9 * (size_t)j, J->aln, 36);
        int mp = J->max_pos;
        ret[j] = or_extend((const or_index_t *)ix, &o, R->n_stacks, J->dir, J->len, codes + J->off, bids + J->off,
                           J->lo, J->n, aln_out + 9 * (size_t)j, &mp);
        max_pos[j] = mp;
    }
    return 0;
}

int hsa_width0_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens, const uint8_t *codes,
                     size_t codes_len, uint32_t *width_out)
{
    (void)codes_len;
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        width_out[o] = width_out[o + 1] = 0;
        or_cal_width0((const or_index_t *)ix, (int)lens[i], codes + offs[i], width_out + o);
        o += 2 * ((size_t)lens[i] + 1);
    }
    return 0;
}

/* hsa_extend_sliced: every call runs to completion here (the budget is an upper bound
 * on the work of one call, so finishing is a valid answer). */
int hsa_extend_sliced(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs,
                      const int32_t *slots, const uint8_t *resume, int n, const uint8_t *codes, const int32_t *bids,
                      size_t win_len, int n_slots, uint32_t budget, int32_t *ret, int32_t *max_pos, uint32_t *aln_out)
{
    (void)slots; (void)resume; (void)n_slots; (void)budget;
    return hsa_extend_batch(ix, regimes, n_regimes, jobs, n, codes, bids, win_len, ret, max_pos, aln_out);
}
