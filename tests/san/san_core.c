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

/* hsa_splice_prefetch_batch (include/hsa_gpu.h) on the restatement: the rows, the six
 * seed calls and the anchors of every read, and the SA lookups of their hits. */
static int32_t *g_pf_rows, *g_pf_n, *g_pf_wa;
static uint64_t *g_pf_hit, *g_pf_sa;
static hv_t g_pf_hits;
static uint32_t *g_pf_sav;
static size_t g_pf_nsa, g_pf_sacap;

int hsa_splice_prefetch_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg, int n,
                              const uint32_t *lens, const uint64_t *offs, const uint8_t *codes, size_t codes_len,
                              const int32_t *anchor_max_diff, hsa_splice_pf_t *out)
{
    (void)codes_len;
    const or_index_t *ox = (const or_index_t *)ix;
    memset(out, 0, sizeof *out);
    free(g_pf_rows); free(g_pf_n); free(g_pf_wa); free(g_pf_hit); free(g_pf_sa); free(g_pf_hits.h); free(g_pf_sav);
    g_pf_hits.h = NULL; g_pf_hits.n = g_pf_hits.cap = 0; g_pf_sav = NULL; g_pf_nsa = g_pf_sacap = 0;
    int M = 0;
    for (int r = 0; r < n; ++r) M = (int)lens[r] > M ? (int)lens[r] : M;
    const size_t rs = (size_t)M + 1, cws = (size_t)(M / 3 + 3 > 13 ? M / 3 + 3 : 13);
    g_pf_rows = (int32_t *)calloc((size_t)n * 6 * rs * 2 + 2, 4);
    g_pf_n = (int32_t *)calloc((size_t)n * 8 + 1, 4);
    g_pf_hit = (uint64_t *)calloc((size_t)n * 8 + 1, 8);
    g_pf_sa = (uint64_t *)calloc((size_t)n * 8 + 1, 8);
    g_pf_wa = (int32_t *)calloc((size_t)n * 8 * cws * 2 + 2, 4);
    uint8_t *ss[2];
    ss[0] = (uint8_t *)malloc((size_t)M + 1);
    ss[1] = (uint8_t *)malloc((size_t)M + 1);
    for (int r = 0; r < n; ++r) {
        const int L = (int)lens[r], sl = L / 3;
        const uint8_t *q = codes + offs[r];
        for (int j = 0; j < L; ++j) { ss[0][j] = q[j]; ss[1][j] = q[L - 1 - j] < 4 ? (uint8_t)(3 - q[L - 1 - j]) : q[L - 1 - j]; }
        int32_t *row[6];
        for (int j = 0; j < 6; ++j) row[j] = g_pf_rows + 2 * ((size_t)r * 6 + (size_t)j) * rs;
        for (int s = 0; s < 2; ++s) {
            or_cal_width(ox, L, ss[s], (uint32_t *)row[s]);
            if (L >= 12) or_cal_width(ox, 12, ss[s] + L - 12, (uint32_t *)row[2 + s]);
            or_cal_width0(ox, L, ss[s], (uint32_t *)row[4 + s]);
        }
        for (int c = 0; c < 8; ++c) {
            const int s = c < 6 ? c / 3 : c - 6, t = c % 3;
            const size_t cc = 8 * (size_t)r + (size_t)c;
            int32_t *cw = g_pf_wa + 2 * cc * cws;
            hsa_job_t J;
            memset(&J, 0, sizeof J);
            const uint8_t *sq;
            int len, kind;
            const hsa_regime_t *R;
            if (c < 6) {
                const int la = sl + (t == 2 ? L % 3 : 0);
                for (int p = 0; p < la; ++p) { cw[2 * p] = row[s][2 * p]; cw[2 * p + 1] = row[s][2 * p + 1]; }
                cw[2 * la] = 0;
                cw[2 * la + 1] = (la ? row[s][2 * (la - 1) + 1] : 0) + 1;
                J.max_diff = seed_rg->max_diff; J.seed_len = la;
                sq = ss[s] + t * sl; len = la; kind = 2; R = seed_rg;
            } else {
                const int32_t *cn = g_pf_n + 8 * (size_t)r + 3 * s;
                const int mask = (cn[0] > 0) | (cn[1] > 0) << 1 | (cn[2] > 0) << 2;
                if (L <= 12 || (mask != 3 && mask != 6)) { g_pf_n[cc] = -1; continue; }
                const int tail = mask == 3;
                const int32_t *src = tail ? row[2 + s] : row[s];
                for (int p = 0; p < 13; ++p) { cw[2 * p] = src[2 * p]; cw[2 * p + 1] = src[2 * p + 1]; }
                J.max_diff = anchor_max_diff[r];
                sq = ss[s] + (tail ? L - 12 : 0); len = 12; kind = 0; R = anchor_rg;
            }
            or_opt_t o = opt_of(R, &J);
            uint32_t *h = NULL;
            const int na = or_match_gap(ox, &o, R->n_stacks, sq, len, s, (uint32_t *)cw, kind, NULL, &h);
            g_pf_n[cc] = na;
            g_pf_hit[cc] = g_pf_hits.n;
            if (na > 0) hv_add(&g_pf_hits, h, na);
            or_free(h);
        }
        if (!g_sa_vals) continue;
        for (int c = 0; c < 8; ++c) {                   /* k .. min(l, k + 49) of every hit */
            const size_t cc = 8 * (size_t)r + (size_t)c;
            g_pf_sa[cc] = g_pf_nsa;
            for (int x = 0; x < g_pf_n[cc]; ++x) {
                const uint32_t *hh = g_pf_hits.h + 9 * (g_pf_hit[cc] + (size_t)x);
                for (uint32_t j = hh[1]; j <= hh[2] && j < hh[1] + 50u; ++j) {
                    if (g_pf_nsa == g_pf_sacap) {
                        g_pf_sacap = g_pf_sacap ? 2 * g_pf_sacap : 1024;
                        g_pf_sav = (uint32_t *)realloc(g_pf_sav, g_pf_sacap * 16);
                    }
                    if (hsa_sa_position_batch(ix, 1, &j, g_pf_sav + 4 * g_pf_nsa)) return HSA_E_ARG;
                    ++g_pf_nsa;
                }
            }
        }
    }
    free(ss[0]); free(ss[1]);
    out->n = n; out->max_len = M; out->row_stride = (int)rs; out->cw_stride = (int)cws;
    out->rows = g_pf_rows; out->call_n = g_pf_n; out->call_hit = g_pf_hit;
    out->hits = g_pf_hits.h ? g_pf_hits.h : (g_pf_hits.h = (uint32_t *)calloc(9, 4));
    out->wafter = g_pf_wa; out->call_sa = g_sa_vals ? g_pf_sa : NULL; out->sa = g_pf_sav;
    out->n_hits = g_pf_hits.n; out->n_sa = g_pf_nsa;
    return 0;
}

/* The splice kernel (hsa_splice.hip) has no restatement here: the sanitized drop-in takes
 * the host's bwt_splice_match for every fallback read, as it does on an index without the
 * packed text. */
int hsa_index_set_text(hsa_index_t *ix, const uint32_t *packed, uint64_t n_words, uint32_t dna_len)
{
    (void)ix; (void)packed; (void)n_words; (void)dna_len;
    return 0;
}

int hsa_splice_match_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                           const hsa_regime_t *ext_rg, int n, const uint32_t *lens, const uint64_t *offs,
                           const uint8_t *codes, size_t codes_len, const int32_t *anchor_max_diff, hsa_splice_pf_t *pf,
                           uint32_t *res, hsa_splice_stats_t *stats)
{
    (void)ix; (void)seed_rg; (void)anchor_rg; (void)ext_rg; (void)n; (void)lens; (void)offs; (void)codes;
    (void)codes_len; (void)anchor_max_diff; (void)pf; (void)res; (void)stats;
    /* SAN_SPLICE_FAKE=1: a "device" whose answers disagree with the host's bwt_splice_match
     * (every read answered, with no hit): the drop-in's guard must notice on the first batch
     * and run the host's function for every fallback read (tests/test_dropin_cpu.py) */
    const char *fk = getenv("SAN_SPLICE_FAKE");
    if (fk && atoi(fk) == 1) {
        memset(res, 0, sizeof(uint32_t) * HSA_SP_RES_WORDS * (size_t)n);
        if (stats) memset(stats, 0, sizeof *stats);
        return 0;
    }
    return HSA_E_ARG;
}
