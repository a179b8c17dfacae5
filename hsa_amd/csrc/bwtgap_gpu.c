/*
 * bwtgap_gpu.c -- host side of the drop-in bwt_match_gap (bwtgap.c:118-331, declared
 * bwtgap.h:26) on the MI355X search core: the calls the host's splice path makes
 * (bwt_splice_match's seed and anchor searches, bwtgap.c:812, :919, :1192), with the
 * caller's widths, width_seed NULL or aliased, and width_back handed back as
 * gap_shadow leaves it.  Its own object so that a host can take the GPU
 * bwa_cal_sa_reg_gap alone (bwtaln_gpu.o) or both entry points.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hsa_bwtaln.h"
#include "bwtaln_gpu.h"

/* capacity of the reference's hit array after n appends: calloc of 10, doubled when
 * full (bwtgap.c:137-138, :218-227); the tail stays zero */
static int aln_capacity(int n)
{
    int m = 10;
    while (m < n) m <<= 1;
    return m;
}

/* The regime of one direct call: its option block and the stack it was given. */
static hsa_regime_t call_regime(const bwt_aux_t *a)
{
    const gap_opt_t *o = a->opt;
    const int n_stacks = a->stack ? a->stack->n_stacks
                                  : hsa_aln_score(o, o->max_diff + 1, o->max_gapo + 1, o->max_gape + 1);
    return hsa_regime_of(o, n_stacks, o->max_diff);
}

static int same_regime(const hsa_regime_t *x, const hsa_regime_t *y)
{
    hsa_regime_t a = *x, b = *y;
    a.max_diff = b.max_diff = 0;            /* the per-call max_diff travels in the job */
    return memcmp(&a, &b, sizeof a) == 0;
}

/* bwt_match_gap (bwtgap.c:118-331) for n independent calls, as the host's callers
 * make them (bwtaln.c:350; bwt_splice_match's seed and anchor searches, bwtgap.c:812,
 * :919, :1192): out[i] is a calloc'd bwt_aln1_t array of the reference's capacity,
 * n_out[i] its hit count, and aux[i]->width_back is updated as gap_shadow leaves it
 * (bwtgap.c:217).  Calls with different options run as separate regimes of one or
 * more launches.  Returns 0, or exits(1) on a GPU failure (the reference's
 * convention). */
int bwt_match_gap_batch(bwt_aux_t *const *aux, int n, bwt_aln1_t **out, int *n_out)
{
    if (n <= 0) return 0;
    hsa_index_t *ix = hsa_gpu_index_of(aux[0]->bi_bwt);
    hsa_gpu_lock();
    hsa_regime_t *rg = (hsa_regime_t *)malloc(sizeof(hsa_regime_t) * (size_t)n);
    int *gid = (int *)malloc(sizeof(int) * (size_t)n);
    int ng = 0;
    for (int i = 0; i < n; ++i) {
        if (aux[i]->bi_bwt != aux[0]->bi_bwt) { fprintf(stderr, "[bwt_match_gap_batch] calls on different indexes\n"); exit(1); }
        hsa_regime_t r = call_regime(aux[i]);
        int g = 0;
        while (g < ng && !same_regime(&rg[g], &r)) ++g;
        if (g == ng) rg[ng++] = r;
        else if (r.max_diff > rg[g].max_diff) rg[g].max_diff = r.max_diff;
        gid[i] = g;
    }
    for (int g0 = 0; g0 < ng; g0 += 2) {     /* two regimes per launch */
        const int nr = ng - g0 < 2 ? ng - g0 : 2;
        int m = 0;
        size_t ncodes = 0, npairs = 0;
        for (int i = 0; i < n; ++i) {
            if (gid[i] < g0 || gid[i] >= g0 + nr) continue;
            const bwt_aux_t *a = aux[i];
            ++m;
            ncodes += (size_t)a->len;
            npairs += (size_t)a->len + 1;
            if (a->width_seed && a->width_seed != a->width_back && a->opt->seed_len > 0)
                npairs += (size_t)a->opt->seed_len + 1;
        }
        hsa_job_t *jobs = (hsa_job_t *)calloc((size_t)m + 1, sizeof(hsa_job_t));
        hsa_mg_job_t *mg = (hsa_mg_job_t *)calloc((size_t)m + 1, sizeof(hsa_mg_job_t));
        int *map = (int *)malloc(sizeof(int) * ((size_t)m + 1));
        uint8_t *codes = (uint8_t *)malloc(ncodes + 1);
        int32_t *w = (int32_t *)malloc(8 * (npairs + 1));
        int32_t *n_aln = (int32_t *)malloc(sizeof(int32_t) * ((size_t)m + 1));
        uint64_t *hoff = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)m + 1));
        size_t co = 0, wo = 0;
        int q = 0;
        for (int i = 0; i < n; ++i) {
            if (gid[i] < g0 || gid[i] >= g0 + nr) continue;
            const bwt_aux_t *a = aux[i];
            const ubyte_t *seq = a->strand == 1 ? a->rc_seq : a->seq;           /* bwtgap.c:123 */
            jobs[q].off = co; jobs[q].len = (uint32_t)a->len; jobs[q].max_diff = a->opt->max_diff;
            jobs[q].seed_len = a->opt->seed_len; jobs[q].regime = gid[i] - g0;
            memcpy(codes + co, seq, (size_t)a->len);
            co += (size_t)a->len;
            mg[q].strand = a->strand;
            mg[q].wb_off = wo;
            memcpy(w + 2 * wo, a->width_back, 8 * ((size_t)a->len + 1));
            wo += (size_t)a->len + 1;
            if (!a->width_seed) {
                mg[q].seed = HSA_SEED_NONE;
            } else if (a->width_seed == a->width_back) {
                mg[q].seed = HSA_SEED_ALIAS;
            } else if (a->opt->seed_len < 0) {
                mg[q].seed = HSA_SEED_NONE;     /* ii < 0 throughout: the seed rows are never read */
            } else {
                mg[q].seed = HSA_SEED_OWN;
                mg[q].ws_off = wo;
                memcpy(w + 2 * wo, a->width_seed, 8 * ((size_t)a->opt->seed_len + 1));
                wo += (size_t)a->opt->seed_len + 1;
            }
            map[q++] = i;
        }
        uint32_t *hits = NULL;
        long tot = hsa_match_gap_batch(ix, rg + g0, nr, jobs, mg, m, codes, ncodes, w, wo, w, n_aln, hoff, &hits, NULL);
        if (tot < 0) hsa_gpu_fatal("GPU bwt_match_gap", tot);
        for (int j = 0; j < m; ++j) {
            bwt_aux_t *a = aux[map[j]];
            bwt_aln1_t *p = (bwt_aln1_t *)calloc((size_t)aln_capacity(n_aln[j]), sizeof(bwt_aln1_t));
            if (n_aln[j] > 0) memcpy(p, hits + hoff[j] * 9, sizeof(bwt_aln1_t) * (size_t)n_aln[j]);
            out[map[j]] = p;
            n_out[map[j]] = n_aln[j];
            memcpy(a->width_back, w + 2 * mg[j].wb_off, 8 * ((size_t)a->len + 1));
        }
        hsa_free(hits);
        free(jobs); free(mg); free(map); free(codes); free(w); free(n_aln); free(hoff);
    }
    free(rg); free(gid);
    hsa_gpu_unlock();
    return 0;
}

/* ------------------------------------------------------------ splice prefetch
 * bwt_splice_match (bwtgap.c:748) asks for its widths, seed searches, anchor searches and
 * SA -> position lookups one call at a time, each a GPU round trip.  Which of them it
 * asks for depends on earlier answers, but everything it can ask for before its first
 * seed extension is determined by its read alone: bwa_cal_sa_reg_gap runs all of that for
 * every fallback read of a batch in one device pass first (hsa_splice_prefetch ->
 * hsa_splice_prefetch_batch, include/hsa_gpu.h) and the entry points answer from the
 * result.  The table is per read: the runner (bwtext_gpu.c) and the serial loop
 * (bwtaln_gpu.c) name the read a thread is working on (hsa_splice_set_read), and a call
 * is answered only by that read's entries, after comparing every input of the call with
 * the entry's -- options, strand, length, the sequence, widths, width_seed kind, the
 * stack's bucket count -- so an answer from the table is the answer the call would
 * compute.  Anything else (a call after an extension, another read's) is searched on its
 * own.  The table is filled before the splice path starts and read-only while it runs: no
 * locks. */
typedef struct {
    int n, n_stacks;
    hsa_splice_pf_t pf;            /* the device pass's outputs (pinned; valid until the next batch) */
    const ubyte_t **seq;           /* per read: the read (strand 0) */
    ubyte_t *rc;                   /* per read: its reverse complement (strand 1), at 2 * max_len * r */
    int *len;
    gap_opt_t *aopt;               /* per read: the anchors' options (bwtgap.c:777-782) */
    gap_opt_t sopt;                /* the seed options without seed_len (bwtgap.c:769-774) */
    const Idx2BWT *bi;
} pf_tab_t;

static pf_tab_t g_pf;
static int g_pf_live;
static __thread int tl_pf_read = -1;
static uint64_t g_memo_hits, g_memo_misses, g_w_hits, g_w_misses, g_sa_hits, g_sa_misses;

/* The fallback read (prefetch order) the calling thread's bwt_splice_match works on, or -1. */
void hsa_splice_set_read(int r) { tl_pf_read = r; }

static const pf_tab_t *tab_of(const Idx2BWT *bi, int *r)
{
    *r = tl_pf_read;
    if (!g_pf_live || *r < 0 || *r >= g_pf.n || bi != g_pf.bi) return NULL;
    return &g_pf;
}

static const ubyte_t *strand_seq(const pf_tab_t *t, int r, int s)
{
    return s ? t->rc + (size_t)2 * (size_t)t->pf.max_len * (size_t)r : t->seq[r];
}

static const int32_t *row_of(const pf_tab_t *t, int r, int j)
{
    return t->pf.rows + 2 * ((size_t)6 * (size_t)r + (size_t)j) * (size_t)t->pf.row_stride;
}

/* width_back[0..n] equals row[0..n) and then {0, bid of row[n - 1] + 1} (a prefix's widths) */
static int same_prefix_widths(const bwt_width_t *w, const int32_t *row, int n)
{
    for (int i = 0; i < n; ++i)
        if ((int32_t)w[i].w != row[2 * i] || w[i].bid != row[2 * i + 1]) return 0;
    return w[n].w == 0 && w[n].bid == (n ? row[2 * (n - 1) + 1] : 0) + 1;
}

static int same_widths(const bwt_width_t *w, const int32_t *row, int n)
{
    for (int i = 0; i < n; ++i)
        if ((int32_t)w[i].w != row[2 * i] || w[i].bid != row[2 * i + 1]) return 0;
    return 1;
}

/* The table's answer to bwt_match_gap(aux), or NULL. */
static bwt_aln1_t *table_match_gap(const bwt_aux_t *aux, int *n_out)
{
    int r;
    const pf_tab_t *t = tab_of(aux->bi_bwt, &r);
    if (!t || !aux->stack || aux->stack->n_stacks != t->n_stacks || (aux->strand != 0 && aux->strand != 1)) return NULL;
    const int s = aux->strand, n = aux->len, L = t->len[r], sl = L / 3;
    const ubyte_t *sq = s ? aux->rc_seq : aux->seq, *ss = strand_seq(t, r, s);
    const int32_t *cn = t->pf.call_n + 8 * (size_t)r;
    int call = -1;
    if (aux->width_seed == aux->width_back) {                 /* a seed (bwtgap.c:797-812) */
        for (int tt = 0; tt < 3 && call < 0; ++tt) {
            const int la = sl + (tt == 2 ? L % 3 : 0), c = 3 * s + tt;
            if (la != n || cn[c] < 0 || memcmp(sq, ss + tt * sl, (size_t)n)) continue;
            gap_opt_t o = t->sopt;
            o.seed_len = la;
            if (memcmp(aux->opt, &o, sizeof o) || !same_prefix_widths(aux->width_back, row_of(t, r, s), la)) continue;
            call = c;
        }
    } else if (!aux->width_seed && n == 12 && cn[6 + s] >= 0) {     /* an anchor (bwtgap.c:911-919, :1187-1192) */
        const int tail = cn[3 * s] > 0 && cn[3 * s + 1] > 0;           /* pattern 3: the last 12 bases */
        if (!memcmp(sq, ss + (tail ? L - 12 : 0), 12) && !memcmp(aux->opt, t->aopt + r, sizeof(gap_opt_t)) &&
            same_widths(aux->width_back, row_of(t, r, tail ? 2 + s : s), 13))
            call = 6 + s;
    }
    if (call < 0) return NULL;
    const size_t c = 8 * (size_t)r + (size_t)call;
    const int na = t->pf.call_n[c];
    bwt_aln1_t *out = (bwt_aln1_t *)calloc((size_t)aln_capacity(na), sizeof(bwt_aln1_t));
    if (na > 0) memcpy(out, t->pf.hits + 9 * t->pf.call_hit[c], sizeof(bwt_aln1_t) * (size_t)na);
    memcpy(aux->width_back, t->pf.wafter + 2 * c * (size_t)t->pf.cw_stride, sizeof(bwt_width_t) * ((size_t)n + 1));
    *n_out = na;
    return out;
}

/* bwt_cal_width (bwtaln.c:73-116) from the calling thread's read's rows: type 1 of any
 * prefix of either strand, or of its last 12 bases; type 0 of the whole strand.  Returns
 * 1 with width and *ret written, 0 when the table does not hold it. */
int hsa_splice_table_width(const Idx2BWT *bi, int len, const ubyte_t *str, bwt_width_t *width, int type, int *ret)
{
    int r;
    const pf_tab_t *t = tab_of(bi, &r);
    if (!t || len < 0) return 0;
    const int L = t->len[r];
    for (int s = 0; s < 2; ++s) {
        const ubyte_t *ss = strand_seq(t, r, s);
        if (type == 1 && len <= L && !memcmp(str, ss, (size_t)len)) {
            const int32_t *row = row_of(t, r, s);
            for (int i = 0; i < len; ++i) { width[i].w = (bwtint_t)row[2 * i]; width[i].bid = row[2 * i + 1]; }
            width[len].w = 0;
            width[len].bid = (len ? row[2 * (len - 1) + 1] : 0) + 1;
            *ret = width[len].bid;
            __atomic_fetch_add(&g_w_hits, 1, __ATOMIC_RELAXED);
            return 1;
        }
        if ((type == 1 && len == 12 && L >= 12 && !memcmp(str, ss + L - 12, 12)) ||
            (type != 1 && len == L && !memcmp(str, ss, (size_t)len))) {
            const int32_t *row = row_of(t, r, type == 1 ? 2 + s : 4 + s);
            for (int i = type == 1 ? 0 : 1; i <= len; ++i) { width[i].w = (bwtint_t)row[2 * i]; width[i].bid = row[2 * i + 1]; }
            *ret = width[len].bid;
            __atomic_fetch_add(&g_w_hits, 1, __ATOMIC_RELAXED);
            return 1;
        }
    }
    __atomic_fetch_add(&g_w_misses, 1, __ATOMIC_RELAXED);
    return 0;
}

/* SA index -> (occ, seq id, 1-based position) for the calling thread's read: the lookups
 * bwt_aln_corelate_check makes on its seed and anchor hits (bwtgap.c:698, :711).
 * Returns 1 with o[0..2] = occ, sid, ori, else 0. */
int hsa_splice_table_sa(const Idx2BWT *bi, uint32_t idx, uint32_t o[3])
{
    int r;
    const pf_tab_t *t = tab_of(bi, &r);
    if (!t || !t->pf.call_sa) return 0;
    for (int c = 0; c < 8; ++c) {
        const size_t cc = 8 * (size_t)r + (size_t)c;
        const int na = t->pf.call_n[cc];
        if (na <= 0) continue;
        const uint32_t *h = t->pf.hits + 9 * t->pf.call_hit[cc];
        uint64_t cur = t->pf.call_sa[cc];
        for (int x = 0; x < na; ++x) {
            const uint32_t k = h[9 * x + 1], l = h[9 * x + 2], lim = k + 50u;
            const uint32_t span = (k > l || lim < k) ? 0u : (l < lim - 1u ? l : lim - 1u) - k + 1u;
            if (idx >= k && idx - k < span) {
                const uint32_t *v = t->pf.sa + 4 * (cur + (idx - k));
                o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
                __atomic_fetch_add(&g_sa_hits, 1, __ATOMIC_RELAXED);
                return 1;
            }
            cur += span;
        }
    }
    __atomic_fetch_add(&g_sa_misses, 1, __ATOMIC_RELAXED);
    return 0;
}

void hsa_splice_memo_clear(void)
{
    g_pf_live = 0;
    free(g_pf.seq); free(g_pf.rc); free(g_pf.len); free(g_pf.aopt);
    memset(&g_pf, 0, sizeof g_pf);
}

/* The prefetch for reads aux[0..n) as bwt_splice_match receives them (seq, rc_seq, len,
 * opt = local_opt of that read, stack with the batch's n_stacks), in the order the splice
 * path will run them (hsa_splice_set_read's numbering). */
static int prefetch_impl(const Idx2BWT *bi, int n, bwt_aux_t *const *aux, int fatal);

int hsa_splice_prefetch(const Idx2BWT *bi, int n, bwt_aux_t *const *aux) { return prefetch_impl(bi, n, aux, 1); }

/* fatal == 0: the attach-time warm-up, whose answers are discarded: a failure (e.g. HBM
 * short at attach) is logged under HSA_VERBOSE and ignored */
static int prefetch_impl(const Idx2BWT *bi, int n, bwt_aux_t *const *aux, int fatal)
{
    hsa_splice_memo_clear();
    if (n <= 0) return 0;
    const double t_start = hsa_now();
    hsa_index_t *ix = hsa_gpu_index_of(bi);
    const gap_opt_t *o0 = aux[0]->opt;
    const int n_stacks = aux[0]->stack ? aux[0]->stack->n_stacks
                                       : hsa_aln_score(o0, o0->max_diff + 1, o0->max_gapo + 1, o0->max_gape + 1);
    int max_len = 0, ok = 1;
    size_t tot = 0;
    for (int r = 0; r < n; ++r) {
        const gap_opt_t *o = aux[r]->opt;
        /* one seed and one anchor regime: every read's options but max_diff / seed_len equal */
        gap_opt_t a = *o, b = *o0;
        a.max_diff = b.max_diff = 0; a.seed_len = b.seed_len = 0;
        if (memcmp(&a, &b, sizeof a) || aux[r]->len < 3 || aux[r]->len > 3 * 1021 ||
            (aux[r]->stack && aux[r]->stack->n_stacks != n_stacks))
            ok = 0;
        if (aux[r]->len > max_len) max_len = aux[r]->len;
        tot += (size_t)aux[r]->len;
    }
    if (!ok) return 0;                     /* no table: every call of the splice path runs on its own */
    pf_tab_t *t = &g_pf;
    t->n = n; t->n_stacks = n_stacks; t->bi = bi;
    t->seq = (const ubyte_t **)malloc(sizeof(ubyte_t *) * (size_t)n);
    t->rc = (ubyte_t *)malloc((size_t)2 * (size_t)max_len * (size_t)n + 16);
    t->len = (int *)malloc(sizeof(int) * (size_t)n);
    t->aopt = (gap_opt_t *)malloc(sizeof(gap_opt_t) * (size_t)n);
    uint32_t *lens = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n);
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    int32_t *amd = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    uint8_t *codes = (uint8_t *)malloc(tot + 1);
    size_t co = 0;
    int amd_max = 0;
    for (int r = 0; r < n; ++r) {
        const bwt_aux_t *a = aux[r];
        const int L = a->len;
        t->seq[r] = a->seq; t->len[r] = L;
        ubyte_t *rc = t->rc + (size_t)2 * (size_t)max_len * (size_t)r;
        for (int j = 0; j < L; ++j) { const ubyte_t c = a->seq[L - 1 - j]; rc[j] = c < 4 ? (ubyte_t)(3 - c) : c; }
        t->aopt[r] = *a->opt;
        t->aopt[r].max_gape = 3;                                /* aux_ext (bwtgap.c:777-782) */
        lens[r] = (uint32_t)L; offs[r] = co; amd[r] = a->opt->max_diff;
        amd_max = amd[r] > amd_max ? amd[r] : amd_max;
        memcpy(codes + co, a->seq, (size_t)L);
        co += (size_t)L;
    }
    t->pf.max_len = max_len;
    t->sopt = *o0;                                              /* aux_seed (bwtgap.c:769-774) */
    t->sopt.mode &= ~BWA_MODE_GAPE;
    t->sopt.max_gapo = 0;
    t->sopt.max_gape = 0;
    t->sopt.max_diff = o0->max_seed_diff;
    gap_opt_t ao = t->aopt[0];
    const hsa_regime_t srg = hsa_regime_of(&t->sopt, n_stacks, t->sopt.max_diff);
    const hsa_regime_t arg = hsa_regime_of(&ao, n_stacks, amd_max);
    hsa_gpu_lock();
    const int rc = hsa_splice_prefetch_batch(ix, &srg, &arg, n, lens, offs, codes, co, amd, &t->pf);
    hsa_gpu_unlock();
    free(lens); free(offs); free(amd); free(codes);
    if (rc == HSA_E_ARG) {             /* options or reads outside the device pass: no table */
        if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] splice prefetch skipped: %s\n", hsa_last_error());
        hsa_splice_memo_clear();
        return 0;
    }
    if (rc && !fatal) {
        if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] splice prefetch warm-up failed (ignored): %s\n", hsa_last_error());
        hsa_splice_memo_clear();
        return 0;
    }
    if (rc) hsa_gpu_fatal("GPU splice prefetch", rc);
    g_pf_live = 1;
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] splice prefetch: %d reads, %.3f s (device pass %.1f ms of kernels)\n", n,
                hsa_now() - t_start, t->pf.kernel_ms);
    return 0;
}

/* One small device pass at attach time: the prefetch's kernels loaded and its buffers
 * made before the first batch (its answers are discarded). */
void hsa_splice_prefetch_warm(const Idx2BWT *bi)
{
    for (int gapo = 0; gapo < 2; ++gapo) {       /* anchors without and with gap opens */
    gap_opt_t o;
    memset(&o, 0, sizeof o);
    o.s_mm = 3; o.s_gapo = 11; o.s_gape = 4; o.max_diff = 4; o.max_gapo = gapo; o.max_gape = 6;   /* gap_init_opt */
    o.max_seed_diff = 2; o.seed_len = 32; o.max_entries = 2000000; o.max_top2 = 30; o.indel_end_skip = 5;
    o.max_del_occ = 10; o.fnr = -1.0f;
    ubyte_t seq[2][100], rc[2][100];
    for (int r = 0; r < 2; ++r)
        for (int j = 0; j < 100; ++j) {
            seq[r][j] = (ubyte_t)((j * 7 + r * 3 + (j >> 3)) & 3);
            rc[r][99 - j] = (ubyte_t)(3 - seq[r][j]);
        }
    gap_stack_t st;
    memset(&st, 0, sizeof st);
    st.n_stacks = hsa_aln_score(&o, o.max_diff + 1, o.max_gapo + 1, o.max_gape + 1);
    bwt_aux_t a[2], *ap[2];
    memset(a, 0, sizeof a);
    for (int r = 0; r < 2; ++r) {
        a[r].bi_bwt = (Idx2BWT *)bi; a[r].seq = seq[r]; a[r].rc_seq = rc[r]; a[r].len = 100; a[r].opt = &o;
        a[r].stack = &st; a[r].max_len = 100;
        ap[r] = a + r;
    }
    prefetch_impl(bi, 2, ap, 0);
    hsa_splice_memo_clear();
    }
}

/* Table statistics since the last call (hits, misses), for logs: bwt_match_gap, then
 * bwt_cal_width and SA -> position (hsa_splice_table_stats). */
void hsa_splice_memo_stats(uint64_t *hits, uint64_t *misses)
{
    *hits = __atomic_exchange_n(&g_memo_hits, 0, __ATOMIC_RELAXED);
    *misses = __atomic_exchange_n(&g_memo_misses, 0, __ATOMIC_RELAXED);
}

void hsa_splice_table_stats(uint64_t *w_hits, uint64_t *w_misses, uint64_t *sa_hits, uint64_t *sa_misses)
{
    *w_hits = __atomic_exchange_n(&g_w_hits, 0, __ATOMIC_RELAXED);
    *w_misses = __atomic_exchange_n(&g_w_misses, 0, __ATOMIC_RELAXED);
    *sa_hits = __atomic_exchange_n(&g_sa_hits, 0, __ATOMIC_RELAXED);
    *sa_misses = __atomic_exchange_n(&g_sa_misses, 0, __ATOMIC_RELAXED);
}

/* bwt_match_gap (bwtgap.c:118, declared bwtgap.h:26): the reference's entry point,
 * one call at a time (a batch of one), or an answer prefetched for the splice path.
 * Same return contract: a calloc'd array, never NULL, freed by the caller. */
bwt_aln1_t *bwt_match_gap(bwt_aux_t *aux, int *_n_aln)
{
    bwt_aln1_t *out = table_match_gap(aux, _n_aln);
    if (out) {
        __atomic_fetch_add(&g_memo_hits, 1, __ATOMIC_RELAXED);
        return out;
    }
    if (g_pf_live) __atomic_fetch_add(&g_memo_misses, 1, __ATOMIC_RELAXED);
    bwt_match_gap_batch(&aux, 1, &out, _n_aln);
    return out;
}

/* This object's own bwt_match_gap, whatever the host's symbol table resolves
 * bwt_match_gap to. */
extern __typeof__(bwt_match_gap) hsa_own_match_gap __attribute__((alias("bwt_match_gap"), visibility("hidden")));

/* Whether the host's bwt_splice_match calls this bwt_match_gap (the host linked
 * bwtgap_gpu.o, or weakened its own): only then does a prefetch pay. */
int hsa_splice_prefetch_active(void)
{
    bwt_aln1_t *(*volatile resolved)(bwt_aux_t *, int *) = bwt_match_gap;
    return resolved == hsa_own_match_gap;
}
