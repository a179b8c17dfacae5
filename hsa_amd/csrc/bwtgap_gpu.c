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
    return 0;
}

/* ------------------------------------------------------------ splice prefetch
 * bwt_splice_match (bwtgap.c:748) asks for its six seed searches one call at a time
 * (bwtgap.c:797-848), each a GPU round trip.  Which seeds it asks for depends on
 * earlier answers, but every seed it can ask for is known in advance: so
 * bwa_cal_sa_reg_gap runs all six of every fallback read in one batch first
 * (hsa_splice_prefetch) and bwt_match_gap answers from that table.  A table entry
 * is keyed by everything the search reads -- index, strand, length, sequence,
 * width_back (and an own width_seed), the width_seed kind, the option block and the
 * stack's bucket count -- and compared in full, so an answer from the table is the
 * answer the search would give.  Any other call (the 12-mer anchors, :919 and
 * :1192) misses and runs on its own. */
typedef struct {
    uint64_t h;
    uint8_t *key;          /* the call's inputs, serialised */
    size_t key_len;
    int n_aln;
    bwt_aln1_t *hits;
    bwt_width_t *wout;     /* width_back after the search */
    int len;
} memo_ent_t;

/* The table is process-global (the reference's host calls bwt_splice_match from one
 * thread, but the entry points may be called from several): every access holds
 * g_memo_mu, and a lookup copies its answer out before releasing it. */
static memo_ent_t *g_memo;
static size_t g_memo_cap, g_memo_n;
static uint64_t g_memo_hits, g_memo_misses;
static pthread_rwlock_t g_memo_mu = PTHREAD_RWLOCK_INITIALIZER;   /* lookups share it */
static hsa_arena_t g_memo_arena;        /* keys, hits and widths of the entries */

static size_t key_of(const bwt_aux_t *a, uint8_t *buf)
{
    const ubyte_t *seq = a->strand == 1 ? a->rc_seq : a->seq;
    const int seed = !a->width_seed ? 0 : a->width_seed == a->width_back ? 2 : 1;
    const int n_stacks = a->stack ? a->stack->n_stacks : -1;
    size_t o = 0;
#define PUT(p, n) do { if (buf) memcpy(buf + o, (p), (n)); o += (n); } while (0)
    PUT(&a->bi_bwt, sizeof a->bi_bwt);
    PUT(&a->strand, 4); PUT(&a->len, 4); PUT(&seed, 4); PUT(&n_stacks, 4);
    PUT(a->opt, sizeof(gap_opt_t));
    PUT(seq, (size_t)a->len);
    PUT(a->width_back, sizeof(bwt_width_t) * ((size_t)a->len + 1));
    if (seed == 1 && a->opt->seed_len >= 0) PUT(a->width_seed, sizeof(bwt_width_t) * ((size_t)a->opt->seed_len + 1));
#undef PUT
    return o;
}

static uint64_t key_hash(const uint8_t *p, size_t n)
{
    /* 8 bytes per step (multiply-rotate), the tail byte by byte */
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 29;
    }
    for (; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
    h ^= h >> 32;
    return h | 1;                          /* 0 marks an empty slot */
}

void hsa_splice_memo_clear(void)
{
    pthread_rwlock_wrlock(&g_memo_mu);
    hsa_arena_free(&g_memo_arena);
    free(g_memo);
    g_memo = NULL;
    g_memo_cap = g_memo_n = 0;
    pthread_rwlock_unlock(&g_memo_mu);
}

static void memo_put(const bwt_aux_t *in, const bwt_width_t *wout, const bwt_aln1_t *hits, int n_aln)
{
    if (2 * (g_memo_n + 1) > g_memo_cap) {     /* grow: open addressing at <= 1/2 load */
        size_t cap = g_memo_cap ? g_memo_cap * 2 : 1024;
        memo_ent_t *t = (memo_ent_t *)calloc(cap, sizeof(memo_ent_t));
        for (size_t i = 0; i < g_memo_cap; ++i) {
            if (!g_memo[i].h) continue;
            size_t j = g_memo[i].h & (cap - 1);
            while (t[j].h) j = (j + 1) & (cap - 1);
            t[j] = g_memo[i];
        }
        free(g_memo);
        g_memo = t;
        g_memo_cap = cap;
    }
    const size_t kl = key_of(in, NULL);
    uint8_t *key = (uint8_t *)hsa_arena_alloc(&g_memo_arena, kl);
    key_of(in, key);
    const uint64_t h = key_hash(key, kl);
    size_t j = h & (g_memo_cap - 1);
    while (g_memo[j].h) {
        if (g_memo[j].h == h && g_memo[j].key_len == kl && !memcmp(g_memo[j].key, key, kl)) return;
        j = (j + 1) & (g_memo_cap - 1);
    }
    memo_ent_t *e = g_memo + j;
    e->h = h; e->key = key; e->key_len = kl; e->n_aln = n_aln; e->len = in->len;
    e->hits = (bwt_aln1_t *)hsa_arena_alloc(&g_memo_arena, sizeof(bwt_aln1_t) * (size_t)(n_aln > 0 ? n_aln : 1));
    if (n_aln > 0) memcpy(e->hits, hits, sizeof(bwt_aln1_t) * (size_t)n_aln);
    e->wout = (bwt_width_t *)hsa_arena_alloc(&g_memo_arena, sizeof(bwt_width_t) * ((size_t)in->len + 1));
    memcpy(e->wout, wout, sizeof(bwt_width_t) * ((size_t)in->len + 1));
    ++g_memo_n;
}

static const memo_ent_t *memo_get(const bwt_aux_t *a)
{
    if (!g_memo_n) return NULL;
    const size_t kl = key_of(a, NULL);
    uint8_t stackbuf[4096];
    uint8_t *key = kl <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(kl);
    key_of(a, key);
    const uint64_t h = key_hash(key, kl);
    const memo_ent_t *hit = NULL;
    for (size_t j = h & (g_memo_cap - 1); g_memo[j].h; j = (j + 1) & (g_memo_cap - 1))
        if (g_memo[j].h == h && g_memo[j].key_len == kl && !memcmp(g_memo[j].key, key, kl)) { hit = g_memo + j; break; }
    if (key != stackbuf) free(key);
    return hit;
}

/* The SA indices the splice path's correlation can look up for the prefetched hits
 * (bwt_aln_corelate_check, bwtgap.c:698 and :711: k .. min(l, k + 49) of each hit),
 * collected for the SA -> position prefetch (hsa_splice_take_sa_list). */
static uint32_t *g_sa_list;
static size_t g_sa_n, g_sa_cap;

static void sa_list_add(const bwt_aln1_t *h, int n)     /* caller holds g_memo_mu */
{
    for (int x = 0; x < n; ++x)
        for (uint64_t j = h[x].k; j <= h[x].l && j < (uint64_t)h[x].k + 50; ++j) {
            if (g_sa_n == g_sa_cap) {
                g_sa_cap = g_sa_cap ? 2 * g_sa_cap : 4096;
                g_sa_list = (uint32_t *)realloc(g_sa_list, sizeof(uint32_t) * g_sa_cap);
            }
            g_sa_list[g_sa_n++] = (uint32_t)j;
        }
}

/* The collected SA indices (ownership passes to the caller, who frees them). */
size_t hsa_splice_take_sa_list(uint32_t **idx)
{
    pthread_rwlock_wrlock(&g_memo_mu);
    *idx = g_sa_list;
    const size_t n = g_sa_n;
    g_sa_list = NULL;
    g_sa_n = g_sa_cap = 0;
    pthread_rwlock_unlock(&g_memo_mu);
    return n;
}

/* Search calls[0..c) in one batch (bwt_match_gap_batch) and put every answer in the
 * table, keyed by the call's inputs: win[i] holds its width_back as it was before the
 * search (calls[i].width_back is a scratch copy the search rewrites; a width_seed
 * aliased to it is re-aliased to win[i]).  n_out[i] receives the hit counts. */
static double g_t_search, g_t_put;   /* prefetch timing (HSA_VERBOSE) */

static void batch_into_memo(bwt_aux_t *calls, int c, bwt_width_t **win, int *n_out)
{
    if (c <= 0) return;
    bwt_aux_t **cp = (bwt_aux_t **)calloc((size_t)c, sizeof(bwt_aux_t *));
    bwt_aln1_t **out = (bwt_aln1_t **)malloc(sizeof(bwt_aln1_t *) * (size_t)c);
    for (int i = 0; i < c; ++i) cp[i] = calls + i;
    const double t0 = hsa_now();
    bwt_match_gap_batch(cp, c, out, n_out);
    const double t1 = hsa_now();
    g_t_search += t1 - t0;
    pthread_rwlock_wrlock(&g_memo_mu);
    for (int i = 0; i < c; ++i) {
        bwt_width_t *after = calls[i].width_back;
        const int alias = calls[i].width_seed == after;
        calls[i].width_back = win[i];
        if (alias) calls[i].width_seed = win[i];
        memo_put(calls + i, after, out[i], n_out[i]);
        sa_list_add(out[i], n_out[i]);
        free(after); free(out[i]);
    }
    pthread_rwlock_unlock(&g_memo_mu);
    g_t_put += hsa_now() - t1;
    free(cp); free(out);
}

/* One call of the batch: aux[r] copied as bwt_splice_match copies it (bwtgap.c:756-759),
 * with its own option block, strand, length, and a scratch width_back initialised from
 * w (n + 1 pairs, kept in win). */
static bwt_aux_t *add_call(bwt_aux_t *calls, gap_opt_t *opts, bwt_width_t **win, int c, const bwt_aux_t *a,
                           const gap_opt_t *o, int strand, int len, const uint32_t *w)
{
    bwt_aux_t *x = calls + c;
    *x = *a;
    opts[c] = *o;
    x->opt = opts + c;
    x->len = len;
    x->strand = strand;
    win[c] = (bwt_width_t *)malloc(sizeof(bwt_width_t) * ((size_t)len + 1));
    memcpy(win[c], w, sizeof(bwt_width_t) * ((size_t)len + 1));
    x->width_back = (bwt_width_t *)malloc(sizeof(bwt_width_t) * ((size_t)len + 1));
    memcpy(x->width_back, win[c], sizeof(bwt_width_t) * ((size_t)len + 1));
    x->width_seed = NULL;
    return x;
}

#define ANCHOR 12   /* the anchor length of bwtgap.c:911 and :1187 */

/* The splice path's searches of each read bwt_splice_match will be called on, run on the
 * GPU as two batches before the host asks for them; aux[r] as bwt_splice_match receives
 * it (seq, rc_seq, len, opt = local_opt of that read, stack).
 *  1. The six seed searches (bwtgap.c:762-812): widths of the strand prefixes
 *     (bwt_cal_width type 1, as :807 computes them), width_seed aliased to width_back.
 *  2. The 12-mer anchor searches made after an extension succeeds (options of aux_ext:
 *     max_gape 3, :782; width_seed NULL):
 *       - seeds 0 and 1 of a strand map and seed 2 does not (seg_mtype 3): the strand's
 *         last 12 bases with their own widths (:911-919);
 *       - seeds 1 and 2 map and seed 0 does not (seg_mtype 6): its first 12 bases with
 *         the whole read's widths (:867/:871, :1187-1192), i.e. the first 13 width
 *         entries of the prefix of length 13.
 *     Whether the host reaches them depends on the seed correlation and the
 *     backtracking, so the anchor of every strand whose seed pattern leads there is
 *     searched: one small search per such strand, where the host would otherwise make a
 *     GPU round trip per call. */
int hsa_splice_prefetch(const Idx2BWT *bi, int n, bwt_aux_t *const *aux)
{
    if (n <= 0) return 0;
    const double t_start = hsa_now();
    g_t_search = g_t_put = 0.0;
    hsa_index_t *ix = hsa_gpu_index_of(bi);
    /* widths: per read, strand s, the prefix of seed_len and of seed_len + len % 3 */
    int nw = 0;
    size_t wcodes = 0;
    for (int r = 0; r < n; ++r) {
        const int L = aux[r]->len, sl = L / 3;
        if (sl < 1) continue;
        nw += 4;
        wcodes += 4 * (size_t)sl + 2 * (size_t)(L % 3);
    }
    if (nw == 0) return 0;
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nw);
    uint32_t *lens = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)nw);
    size_t *woff = (size_t *)malloc(sizeof(size_t) * (size_t)nw);
    uint8_t *codes = (uint8_t *)malloc(wcodes + 1);
    size_t co = 0, wo = 0;
    int q = 0;
    for (int r = 0; r < n; ++r) {
        const int L = aux[r]->len, sl = L / 3;
        if (sl < 1) continue;
        for (int s = 0; s < 2; ++s)
            for (int k = 0; k < 2; ++k) {
                const int la = sl + (k ? L % 3 : 0);
                offs[q] = co; lens[q] = (uint32_t)la; woff[q] = wo;
                memcpy(codes + co, s ? aux[r]->rc_seq : aux[r]->seq, (size_t)la);
                co += (size_t)la;
                wo += 2 * ((size_t)la + 1);
                ++q;
            }
    }
    uint32_t *wout = (uint32_t *)malloc(sizeof(uint32_t) * (wo + 2));
    int rc = hsa_width_batch(ix, (size_t)nw, offs, lens, codes, co, wout);
    if (rc) hsa_gpu_fatal("GPU bwt_cal_width", rc);
    /* the seed calls, set up as bwtgap.c:797-810 sets up aux_seed */
    const int nc = 6 * (nw / 4);
    bwt_aux_t *calls = (bwt_aux_t *)calloc((size_t)nc, sizeof(bwt_aux_t));
    gap_opt_t *opts = (gap_opt_t *)malloc(sizeof(gap_opt_t) * (size_t)nc);
    bwt_width_t **win = (bwt_width_t **)malloc(sizeof(bwt_width_t *) * (size_t)nc);
    int *n_out = (int *)malloc(sizeof(int) * (size_t)nc);
    int c = 0, w = 0;
    for (int r = 0; r < n; ++r) {
        const bwt_aux_t *a = aux[r];
        const int L = a->len, sl = L / 3;
        if (sl < 1) continue;
        gap_opt_t so = *a->opt;                                 /* :769-774 */
        so.mode &= ~BWA_MODE_GAPE;
        so.max_gapo = 0;
        so.max_gape = 0;
        so.max_diff = a->opt->max_seed_diff;
        for (int i = 0; i < 6; ++i) {
            const int s = i / 3, la = sl + (i % 3 == 2 ? L % 3 : 0);
            so.seed_len = la;                                   /* :802 */
            const uint32_t *wk = wout + woff[w + 2 * s + (i % 3 == 2 && L % 3 ? 1 : 0)];
            bwt_aux_t *x = add_call(calls, opts, win, c, a, &so, s, la, wk);
            if (s) x->rc_seq = a->rc_seq + (i % 3) * sl;       /* :805-806 */
            else x->seq = a->seq + (i % 3) * sl;
            x->width_seed = x->width_back;                      /* :804-809 */
            ++c;
        }
        w += 4;
    }
    batch_into_memo(calls, c, win, n_out);

    /* the anchors of the strands whose seed pattern is 3 or 6 */
    int na = 0;
    size_t acodes = 0;
    for (int r = 0, rr = 0; r < n; ++r) {
        const int L = aux[r]->len;
        if (L / 3 < 1) continue;
        for (int s = 0; s < 2 && L > ANCHOR; ++s) {
            const int *no = n_out + 6 * rr + 3 * s;
            const int mask = (no[0] > 0) | (no[1] > 0) << 1 | (no[2] > 0) << 2;
            if (mask == 3) { ++na; acodes += ANCHOR; }
            if (mask == 6) { ++na; acodes += ANCHOR + 1; }
        }
        ++rr;
    }
    if (na > 0) {
        uint64_t *ao = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)na);
        uint32_t *al = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)na);
        uint8_t *ac = (uint8_t *)malloc(acodes + 1);
        int *ar = (int *)malloc(sizeof(int) * (size_t)na);     /* read, strand, kind */
        size_t aco = 0, awo = 0;
        int k = 0;
        for (int r = 0, rr = 0; r < n; ++r) {
            const bwt_aux_t *a = aux[r];
            const int L = a->len;
            if (L / 3 < 1) continue;
            for (int s = 0; s < 2 && L > ANCHOR; ++s) {
                const int *no = n_out + 6 * rr + 3 * s;
                const int mask = (no[0] > 0) | (no[1] > 0) << 1 | (no[2] > 0) << 2;
                if (mask != 3 && mask != 6) continue;
                const ubyte_t *sq = s ? a->rc_seq : a->seq;
                const int tail = mask == 3;
                al[k] = tail ? ANCHOR : ANCHOR + 1;
                ao[k] = aco;
                memcpy(ac + aco, tail ? sq + L - ANCHOR : sq, al[k]);
                aco += al[k];
                awo += 2 * ((size_t)al[k] + 1);
                ar[k] = r << 2 | s << 1 | tail;
                ++k;
            }
            ++rr;
        }
        uint32_t *aw = (uint32_t *)malloc(sizeof(uint32_t) * (awo + 2));
        rc = hsa_width_batch(ix, (size_t)na, ao, al, ac, aco, aw);
        if (rc) hsa_gpu_fatal("GPU bwt_cal_width", rc);
        bwt_aux_t *acalls = (bwt_aux_t *)calloc((size_t)na, sizeof(bwt_aux_t));
        gap_opt_t *aopts = (gap_opt_t *)malloc(sizeof(gap_opt_t) * (size_t)na);
        bwt_width_t **awin = (bwt_width_t **)malloc(sizeof(bwt_width_t *) * (size_t)na);
        int *an = (int *)malloc(sizeof(int) * (size_t)na);
        size_t wp = 0;
        for (int j = 0; j < na; ++j) {
            const bwt_aux_t *a = aux[ar[j] >> 2];
            const int s = (ar[j] >> 1) & 1, tail = ar[j] & 1, L = a->len;
            gap_opt_t eo = *a->opt;
            eo.max_gape = 3;                                    /* aux_ext (:777-782) */
            bwt_aux_t *x = add_call(acalls, aopts, awin, j, a, &eo, s, ANCHOR, aw + wp);
            if (tail) {                                         /* :912 */
                if (s) x->rc_seq = a->rc_seq + L - ANCHOR;
                else x->seq = a->seq + L - ANCHOR;
            }
            wp += 2 * ((size_t)al[j] + 1);
        }
        batch_into_memo(acalls, na, awin, an);
        for (int j = 0; j < na; ++j) free(awin[j]);
        free(ao); free(al); free(ac); free(ar); free(aw); free(acalls); free(aopts); free(awin); free(an);
    }
    for (int i = 0; i < c; ++i) free(win[i]);
    free(offs); free(lens); free(woff); free(codes); free(wout);
    free(calls); free(opts); free(win); free(n_out);
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] seed/anchor prefetch: %.3f s (GPU searches %.3f s, table %.3f s, the rest: set-up and "
                        "widths)\n", hsa_now() - t_start, g_t_search, g_t_put);
    return 0;
}

/* Table statistics since the last call (hits, misses), for logs. */
void hsa_splice_memo_stats(uint64_t *hits, uint64_t *misses)
{
    pthread_rwlock_wrlock(&g_memo_mu);
    *hits = g_memo_hits; *misses = g_memo_misses;
    g_memo_hits = g_memo_misses = 0;
    pthread_rwlock_unlock(&g_memo_mu);
}

/* bwt_match_gap (bwtgap.c:118, declared bwtgap.h:26): the reference's entry point,
 * one call at a time (a batch of one), or an answer prefetched for the splice path.
 * Same return contract: a calloc'd array, never NULL, freed by the caller. */
bwt_aln1_t *bwt_match_gap(bwt_aux_t *aux, int *_n_aln)
{
    pthread_rwlock_rdlock(&g_memo_mu);
    const memo_ent_t *e = memo_get(aux);
    if (e) {
        __atomic_fetch_add(&g_memo_hits, 1, __ATOMIC_RELAXED);
        bwt_aln1_t *out = (bwt_aln1_t *)calloc((size_t)aln_capacity(e->n_aln), sizeof(bwt_aln1_t));
        if (e->n_aln > 0) memcpy(out, e->hits, sizeof(bwt_aln1_t) * (size_t)e->n_aln);
        memcpy(aux->width_back, e->wout, sizeof(bwt_width_t) * ((size_t)e->len + 1));
        *_n_aln = e->n_aln;
        pthread_rwlock_unlock(&g_memo_mu);
        return out;
    }
    if (g_memo_n) __atomic_fetch_add(&g_memo_misses, 1, __ATOMIC_RELAXED);
    pthread_rwlock_unlock(&g_memo_mu);
    bwt_aln1_t *out = NULL;
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
