/*
 * bwtaln_gpu.c -- host side of the drop-in: bwa_cal_sa_reg_gap (bwtaln.c:246-417)
 * on top of the MI355X search core (hsa_gpu.h).
 *
 * What stays on the host is the part of bwa_cal_sa_reg_gap that is sequential by
 * construction and costs O(read length): the option-block side effects, the two
 * read filters, and the choice of option regime per read.  The searches
 * themselves (widths + bwt_match_gap on both strands) run on the GPU.
 *
 * The option regimes.  The reference copies local_opt = *opt
 * (:254) BEFORE clearing BWA_MODE_GAPE through aux->opt (:261), writes per-read
 * max_diff/seed_len through aux->opt (:330-332), and after the first read that
 * falls back to splicing points aux->opt at local_opt for the rest of the call
 * (:363).  So a call runs reads [0, f] with regime A (the caller's block) and
 * reads (f, n) with regime B (local_opt), f being the first fallback read.  f is
 * only known after searching, hence: search a first chunk in regime A, find f,
 * search the rest in regime B.  When the two regimes cannot differ for any read
 * (same effective options, equal read lengths) the whole call is one launch.
 */
#include <malloc.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/hsa_bwtaln.h"
#include "bwtaln_gpu.h"

#pragma weak hsa_splice_prefetch_active
#pragma weak hsa_splice_prefetch
#pragma weak hsa_splice_memo_clear
#pragma weak hsa_splice_memo_stats
#pragma weak hsa_splice_extend_active
#pragma weak hsa_splice_run
#pragma weak hsa_splice_table_stats
#pragma weak hsa_splice_set_read
#pragma weak hsa_splice_warm
#pragma weak hsa_splice_prefetch_warm
#pragma weak hsa_splice_sa_clear
#pragma weak hsa_splice_sa_stats

_Static_assert(sizeof(bwt_aln1_t) == 36, "bwt_aln1_t layout");
_Static_assert(sizeof(gap_opt_t) == 64, "gap_opt_t layout");
_Static_assert(sizeof(bwa_seq_t) == 208, "bwa_seq_t layout");
_Static_assert(sizeof(bwt_aux_t) == 96, "bwt_aux_t layout");
_Static_assert(sizeof(BWT) == 128, "BWT layout");
_Static_assert(sizeof(Idx2BWT) == 544, "Idx2BWT layout");
_Static_assert(sizeof(gap_entry_t) == 28, "gap_entry_t layout");
_Static_assert(sizeof(HSP) == 48, "HSP layout");
_Static_assert(sizeof(ChrBlock) == 16, "ChrBlock layout");

#define BWA_AVG_ERR 0.02
#define SEED_NONE 0x7fffffff
#define CHUNK0 8192

/* bwa_cal_maxdiff (bwtaln.c:46-58) */
static int cal_maxdiff(int l, double err, double thres)
{
    double elambda = exp(-l * err);
    double sum, y = 1.0;
    int k, x = 1;
    for (k = 1, sum = elambda; k < 1000; ++k) {
        y *= l * err;
        x *= k;
        sum += elambda * y / x;
        if (1.0 - sum < thres) return k;
    }
    return 2;
}

int hsa_aln_score(const gap_opt_t *o, int m, int g, int e) { return m * o->s_mm + g * o->s_gapo + e * o->s_gape; }

hsa_regime_t hsa_regime_of(const gap_opt_t *o, int n_stacks, int max_diff)
{
    hsa_regime_t r;
    memset(&r, 0, sizeof r);
    r.s_mm = o->s_mm; r.s_gapo = o->s_gapo; r.s_gape = o->s_gape;
    r.mode = o->mode & (BWA_MODE_GAPE | BWA_MODE_LOGGAP | BWA_MODE_NONSTOP);
    /* without gap opens no entry ever leaves state M: GAPE and LOGGAP are inert */
    if (o->max_gapo == 0) r.mode &= ~(BWA_MODE_GAPE | BWA_MODE_LOGGAP);
    r.indel_end_skip = o->indel_end_skip; r.max_del_occ = o->max_del_occ; r.max_entries = o->max_entries;
    r.max_gapo = o->max_gapo; r.max_gape = o->max_gape;
    r.max_seed_diff = o->max_seed_diff; r.max_top2 = o->max_top2;
    r.n_stacks = n_stacks;
    r.max_diff = max_diff;
    return r;
}

/* The mutable option fields the per-read loop reads and writes. */
typedef struct { int opt_max_diff, opt_seed, loc_max_diff, loc_seed; } optstate_t;

enum { K_JOB = 0, K_NFILTER = 1, K_POLYAT = 2 };

/* What the prologue's filters read of a read (bwtaln.c:314-325), computed once per
 * read: its count of codes > 3 (N), and whether its first 15 codes are all 0 or all 3. */
typedef struct { int32_t n_n; int8_t polyat; } readinfo_t;

static readinfo_t read_info(const uint8_t *seq, int len)
{
    readinfo_t ri = {0, 0};
    int j = 0;
    /* 8 codes at a time: a code is > 3 iff one of its bits 2..7 is set */
    for (; j + 8 <= len; j += 8) {
        uint64_t w;
        memcpy(&w, seq + j, 8);
        const uint64_t t = (w >> 2) & 0x3F3F3F3F3F3F3F3Full;
        ri.n_n += __builtin_popcountll(((t + 0x7F7F7F7F7F7F7F7Full) | t) & 0x8080808080808080ull);
    }
    for (; j < len; ++j) ri.n_n += seq[j] > 3;
    if (len >= 15) {
        int a = 1, t = 1;
        for (int k = 0; k < 15; ++k) { a &= seq[k] == 0; t &= seq[k] == 3; }
        ri.polyat = (int8_t)(a || t);
    }
    return ri;
}

/* read_info of reads [r0, r1), a host thread's share */
typedef struct { const uint8_t *codes; const uint64_t *offs; const uint32_t *lens; readinfo_t *ri; int r0, r1; } ri_part_t;

static void *ri_run(void *arg)
{
    ri_part_t *p = (ri_part_t *)arg;
    for (int r = p->r0; r < p->r1; ++r) p->ri[r] = read_info(p->codes + p->offs[r], (int)p->lens[r]);
    return NULL;
}

/* read_info of every read, on up to 8 host threads for large calls */
static void read_infos(const uint8_t *codes, const uint64_t *offs, const uint32_t *lens, int n, readinfo_t *ri)
{
    enum { MAXT = 8 };
    const int nt = n >= (1 << 16) ? MAXT : 1;
    ri_part_t part[MAXT];
    pthread_t th[MAXT];
    int started[MAXT] = {0};
    for (int k = 0; k < nt; ++k) {
        part[k] = (ri_part_t){codes, offs, lens, ri, (int)((long)n * k / nt), (int)((long)n * (k + 1) / nt)};
        if (k > 0) started[k] = pthread_create(&th[k], NULL, ri_run, &part[k]) == 0;
        if (k > 0 && !started[k]) ri_run(&part[k]);
    }
    ri_run(&part[0]);
    for (int k = 1; k < nt; ++k) if (started[k]) pthread_join(th[k], NULL);
}

/* The per-read outputs of the reads the search settled (bwtaln.c:314-373): a read's own
 * calloc'd aln array (capacity >= 10, as bwt_match_gap's) with its hits, the fields
 * cleared; reads [r0, r1), a host thread's share. */
typedef struct {
    bwa_seq_t *seqs; const int32_t *n_aln; const uint32_t *flags; const uint64_t *hoff; const uint32_t *hits;
    int r0, r1;
} out_part_t;

static void *out_run(void *arg)
{
    const out_part_t *o = (const out_part_t *)arg;
    for (int i = o->r0; i < o->r1; ++i) {
        bwa_seq_t *p = o->seqs + i;
        if (o->flags[i] & HSA_RF_NFILTER) continue;             /* untouched (:314-317) */
        p->sa = 0; p->type = 0; p->c1 = p->c2 = 0; p->n_aln = 0; p->aln = 0;
        if ((o->flags[i] & HSA_RF_POLYAT) || o->n_aln[i] <= 0) continue;
        const int cap = o->n_aln[i] > 10 ? o->n_aln[i] : 10;    /* bwt_match_gap's calloc'd array */
        p->aln = (bwt_aln1_t *)calloc(cap, sizeof(bwt_aln1_t));
        memcpy(p->aln, o->hits + o->hoff[i] * 9, sizeof(bwt_aln1_t) * o->n_aln[i]);
        p->n_aln = o->n_aln[i];
    }
    return NULL;
}

/* out_run over every read, on the calling thread: the arrays then come from its heap
 * arena, where the host frees them and the next batch reuses them (on several threads
 * they were slower: allocations from several arenas, freed from the host's) */
static void write_outputs(bwa_seq_t *seqs, int n, const int32_t *n_aln, const uint32_t *flags, const uint64_t *hoff,
                          const uint32_t *hits)
{
    out_part_t part = {seqs, n_aln, flags, hoff, hits, 0, n};
    out_run(&part);
}

/* The splice prefetch of one batch on a thread of its own (bwa_cal_sa_reg_gap). */
typedef struct {
    const Idx2BWT *bi;
    int n;
    bwt_aux_t *fa, **fp;
    gap_opt_t *fo;
    ubyte_t *rc;
    gap_stack_t st_shape;
    double secs;
} pf_job_t;

static void *pf_job_run(void *arg)
{
    pf_job_t *j = (pf_job_t *)arg;
    const double t0 = hsa_now();
    hsa_splice_prefetch(j->bi, j->n, j->fp);
    j->secs = hsa_now() - t0;
    return NULL;
}

/* The prefetch job of reads idx[0..n) as bwt_splice_match receives them (aux of read i:
 * seq, rc_seq, len, local_opt with the read's max_diff / seed_len, the batch's stack). */
static void pf_job_init(pf_job_t *pj, const Idx2BWT *bi, struct bwt_array_t *arr, const bwa_seq_t *seqs,
                        const uint64_t *offs, size_t tot, int max_len, const int *idx, int n, const gap_opt_t *local,
                        const int32_t *sp, int n_stacks)
{
    memset(pj, 0, sizeof *pj);
    pj->bi = bi;
    pj->n = n;
    pj->fa = (bwt_aux_t *)calloc((size_t)n, sizeof(bwt_aux_t));
    pj->fp = (bwt_aux_t **)malloc(sizeof(bwt_aux_t *) * (size_t)n);
    pj->fo = (gap_opt_t *)malloc(sizeof(gap_opt_t) * (size_t)n);
    pj->rc = (ubyte_t *)malloc(tot + 1);
    pj->st_shape.n_stacks = n_stacks;                /* only n_stacks is read */
    for (int q = 0; q < n; ++q) {
        const int i = idx[q];
        const bwa_seq_t *p = seqs + i;
        ubyte_t *r = pj->rc + offs[i];
        for (int j = 0; j < (int)p->len; ++j) {
            ubyte_t c = p->seq[p->len - 1 - j];
            r[j] = c < 4 ? (ubyte_t)(3 - c) : c;
        }
        pj->fo[q] = *local;
        pj->fo[q].max_diff = sp[2 * i];
        pj->fo[q].seed_len = sp[2 * i + 1];
        bwt_aux_t *x = pj->fa + q;
        x->bi_bwt = (Idx2BWT *)bi; x->arr = arr; x->max_len = max_len;
        x->seq = p->seq; x->rc_seq = r; x->len = (int)p->len; x->opt = pj->fo + q;
        x->stack = &pj->st_shape;
        pj->fp[q] = x;
    }
}

static void pf_job_free(pf_job_t *pj) { free(pj->fa); free(pj->fp); free(pj->fo); free(pj->rc); }

/* bwt_splice_match of a batch's fallback reads on the device (hsa_splice_match_batch). */
typedef struct {
    hsa_index_t *ix;
    int n;
    const int *fb;                   /* the reads, in order */
    const bwa_seq_t *seqs;
    const int32_t *sp;               /* per read: local_opt's max_diff, seed_len */
    gap_opt_t local;
    int n_stacks;
    uint32_t *res;                   /* HSA_SP_RES_WORDS per read */
    int lock;                        /* slot 0: its index is shared with direct calls (hsa_gpu_lock) */
    int rc;
    double secs;
    hsa_splice_stats_t st;
} dsp_job_t;

static void *dsp_job_run(void *arg)
{
    dsp_job_t *j = (dsp_job_t *)arg;
    const double t0 = hsa_now();
    uint32_t *lens = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)j->n);
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)j->n);
    int32_t *amd = (int32_t *)malloc(sizeof(int32_t) * (size_t)j->n);
    size_t tot = 0;
    int amd_max = 0;
    for (int k = 0; k < j->n; ++k) {
        const bwa_seq_t *p = j->seqs + j->fb[k];
        lens[k] = p->len; offs[k] = tot; tot += p->len;
        amd[k] = j->sp[2 * j->fb[k]];
        amd_max = amd[k] > amd_max ? amd[k] : amd_max;
    }
    uint8_t *codes = (uint8_t *)malloc(tot + 1);
    for (int k = 0; k < j->n; ++k) memcpy(codes + offs[k], j->seqs[j->fb[k]].seq, lens[k]);
    /* aux_seed (bwtgap.c:769-774), aux_ext (:776-782) */
    gap_opt_t so = j->local, ao = j->local;
    so.mode &= ~BWA_MODE_GAPE; so.max_gapo = 0; so.max_gape = 0; so.max_diff = j->local.max_seed_diff;
    ao.max_gape = 3;
    const hsa_regime_t srg = hsa_regime_of(&so, j->n_stacks, so.max_diff);
    const hsa_regime_t arg_ = hsa_regime_of(&ao, j->n_stacks, amd_max);
    hsa_regime_t erg = arg_;
    erg.mode = ao.mode & (BWA_MODE_GAPE | BWA_MODE_LOGGAP | BWA_MODE_NONSTOP);   /* as the extension reads it */
    hsa_splice_pf_t pf;
    if (j->lock) hsa_gpu_lock();
    j->rc = hsa_splice_match_batch(j->ix, &srg, &arg_, &erg, j->n, lens, offs, codes, tot, amd, &pf, j->res, &j->st);
    if (j->lock) hsa_gpu_unlock();
    free(lens); free(offs); free(amd); free(codes);
    j->secs = hsa_now() - t0;
    return NULL;
}

/* One read of the bwtaln.c:303-337 prologue under regime `cur` (0 = A, 1 = B). */
static int plan_read(const gap_opt_t *caller, int cur, optstate_t *st, const readinfo_t *ri, int len,
                     int32_t *max_diff, int32_t *seed_len)
{
    if (ri->n_n > st->loc_max_diff) return K_NFILTER;                  /* :314-317 */
    if (ri->polyat) return K_POLYAT;                                    /* :324-325 */
    int *md = cur ? &st->loc_max_diff : &st->opt_max_diff;
    int *sl = cur ? &st->loc_seed : &st->opt_seed;
    if (caller->fnr > 0.0) *md = cal_maxdiff(len, BWA_AVG_ERR, caller->fnr);   /* :330-331 */
    *sl = st->opt_seed < len ? st->opt_seed : SEED_NONE;                       /* :332 */
    *max_diff = *md;
    *seed_len = *sl;
    return K_JOB;
}

typedef struct {
    uint32_t *h; size_t n, cap;
} hitbuf_t;

static int hb_append(hitbuf_t *b, const uint32_t *src, size_t n)
{
    if (n == 0) return 0;
    if (b->n + n > b->cap) {
        size_t c = (b->n + n) * 2 + 64;
        uint32_t *p = (uint32_t *)realloc(b->h, c * 36);
        if (!p) return -1;
        b->h = p; b->cap = c;
    }
    memcpy(b->h + b->n * 9, src, n * 36);
    b->n += n;
    return 0;
}

/* One device slot's share of a search_range call (its own thread, its own index). */
typedef struct {
    hsa_index_t *ix;
    const hsa_regime_t *rg;
    hsa_job_t *jobs;
    int n;
    const uint8_t *codes;
    size_t codes_len;
    int32_t *na;
    uint32_t *fl;
    uint64_t *ho;
    uint32_t *hits;
    long tot;
    hsa_stats_t st;
    char err[256];
} slot_part_t;

static void *slot_run(void *arg)
{
    slot_part_t *p = (slot_part_t *)arg;
    p->tot = hsa_search_batch(p->ix, p->rg, 1, p->jobs, p->n, p->codes, p->codes_len, p->na, p->fl, p->ho,
                              &p->hits, &p->st);
    if (p->tot < 0) snprintf(p->err, sizeof p->err, "%s", hsa_last_error());
    return NULL;
}

/* Search the reads [r0, r1) whose kind is K_JOB; results into the per-read outputs.
 * With several device slots the jobs are split into contiguous parts, one per slot,
 * searched concurrently (one host thread per slot); reads are independent, so the
 * parts' results are those of one search over all of them. */
static int search_range(hsa_index_t *const *ixs, int n_ix, const hsa_regime_t *rg, int r0, int r1, const int8_t *kind,
                        const int32_t *jmd, const int32_t *jsl, int regime, const uint32_t *lens, const uint64_t *offs,
                        const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                        hitbuf_t *hb, hsa_stats_t *stats)
{
    (void)codes_len;
    int n = 0;
    for (int r = r0; r < r1; ++r) n += kind[r] == K_JOB;
    if (n == 0) return 0;
    if (n == r1 - r0 && n_ix == 1 && hb->n == 0 && !hb->h) {
        /* every read is a job, one slot, no hits yet: the search writes the outputs in place */
        hsa_job_t *jobs = (hsa_job_t *)malloc(sizeof(hsa_job_t) * (size_t)n);
        for (int q = 0; q < n; ++q) {
            const int r = r0 + q;
            jobs[q].off = offs[r] - offs[r0]; jobs[q].len = lens[r]; jobs[q].max_diff = jmd[r]; jobs[q].seed_len = jsl[r];
            jobs[q].regime = 0;
        }
        /* the range's codes: from its lowest offset to its highest read end (the caller's
         * offsets need not ascend; hsa_cal_sa_reg_gap_multi checked every read's bounds) */
        uint64_t c0 = offs[r0], c1 = 0;
        for (int r = r0; r < r1; ++r) {
            if (offs[r] < c0) c0 = offs[r];
            if (offs[r] + lens[r] > c1) c1 = offs[r] + lens[r];
        }
        for (int q = 0; q < n; ++q) jobs[q].off = offs[r0 + q] - c0;
        hsa_stats_t st;
        uint32_t *h = NULL;
        const long tot = hsa_search_batch(ixs[0], rg + regime, 1, jobs, n, codes + c0, (size_t)(c1 - c0),
                                          n_aln + r0, flags + r0, hit_off + r0, &h, &st);
        free(jobs);
        if (tot < 0) return (int)tot;
        hb->h = h; hb->n = hb->cap = (size_t)tot;
        if (stats) {
            stats->rank_queries += st.rank_queries; stats->blocks_loaded += st.blocks_loaded; stats->pops += st.pops;
            stats->overflow_reruns += st.overflow_reruns; stats->kernel_ms += st.kernel_ms;
            stats->main_kernel_ms += st.main_kernel_ms; stats->main_launches += st.main_launches;
        }
        return 0;
    }
    hsa_job_t *jobs = (hsa_job_t *)malloc(sizeof(hsa_job_t) * n);
    int *map = (int *)malloc(sizeof(int) * n);
    int32_t *na = (int32_t *)malloc(sizeof(int32_t) * n);
    uint32_t *fl = (uint32_t *)malloc(sizeof(uint32_t) * n);
    uint64_t *ho = (uint64_t *)malloc(sizeof(uint64_t) * n);
    int q = 0;
    for (int r = r0; r < r1; ++r) {
        if (kind[r] != K_JOB) continue;
        jobs[q].off = offs[r]; jobs[q].len = lens[r]; jobs[q].max_diff = jmd[r]; jobs[q].seed_len = jsl[r];
        jobs[q].regime = 0;
        map[q++] = r;
    }
    if (n_ix < 1) n_ix = 1;
    if (n_ix > n) n_ix = n;
    slot_part_t part[HSA_MAX_SLOTS];
    pthread_t th[HSA_MAX_SLOTS];
    int started[HSA_MAX_SLOTS];
    for (int k = 0; k < n_ix; ++k) {
        const int j0 = (int)((long)n * k / n_ix), j1 = (int)((long)n * (k + 1) / n_ix);
        slot_part_t *p = &part[k];
        memset(p, 0, sizeof *p);
        p->ix = ixs[k]; p->rg = rg + regime; p->jobs = jobs + j0; p->n = j1 - j0;
        p->na = na + j0; p->fl = fl + j0; p->ho = ho + j0;
        /* the part's codes only: offsets rebased to its lowest one */
        uint64_t c0 = jobs[j0].off, c1 = 0;
        for (int j = j0; j < j1; ++j) {
            if (jobs[j].off < c0) c0 = jobs[j].off;
            if (jobs[j].off + jobs[j].len > c1) c1 = jobs[j].off + jobs[j].len;
        }
        for (int j = j0; j < j1; ++j) jobs[j].off -= c0;
        p->codes = codes + c0; p->codes_len = (size_t)(c1 - c0);
        started[k] = k > 0 && pthread_create(&th[k], NULL, slot_run, p) == 0;
        if (k > 0 && !started[k]) slot_run(p);          /* no thread: run it here */
    }
    slot_run(&part[0]);
    for (int k = 1; k < n_ix; ++k) if (started[k]) pthread_join(th[k], NULL);
    int rc = 0;
    for (int k = 0; k < n_ix && rc == 0; ++k)
        if (part[k].tot < 0) { rc = (int)part[k].tot; hsa_gpu_set_error_text(part[k].err); }
    for (int k = 0; k < n_ix && rc == 0; ++k) {
        slot_part_t *p = &part[k];
        const size_t base = hb->n;
        if (hb->n == 0 && !hb->h && n_ix == 1) {       /* the first part's hits: take the array itself */
            hb->h = p->hits; hb->n = hb->cap = (size_t)p->tot;
            p->hits = NULL;
        } else if (hb_append(hb, p->hits, (size_t)p->tot)) { rc = HSA_E_MEM; break; }
        for (int j = 0; j < p->n; ++j) {
            const int r = map[(p->jobs - jobs) + j];
            n_aln[r] = p->na[j]; flags[r] = p->fl[j]; hit_off[r] = p->ho[j] + base;
        }
        if (stats) {
            stats->rank_queries += p->st.rank_queries; stats->blocks_loaded += p->st.blocks_loaded;
            stats->pops += p->st.pops; stats->overflow_reruns += p->st.overflow_reruns;
            stats->kernel_ms += p->st.kernel_ms; stats->main_kernel_ms += p->st.main_kernel_ms;
            stats->main_launches += p->st.main_launches;
        }
    }
    for (int k = 0; k < n_ix; ++k) if (part[k].hits) hsa_free(part[k].hits);
    free(jobs); free(map); free(na); free(fl); free(ho);
    return rc;
}

long hsa_cal_sa_reg_gap_flat(hsa_index_t *ix, gap_opt_t *opt, int n, const uint32_t *lens, const uint64_t *offs,
                             const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                             uint64_t *hit_off, uint32_t **hits, int32_t *splice_opt, hsa_stats_t *stats)
{
    return hsa_cal_sa_reg_gap_multi(&ix, 1, opt, n, lens, offs, codes, codes_len, n_aln, flags, hit_off, hits, splice_opt,
                                    stats);
}

long hsa_cal_sa_reg_gap_multi(hsa_index_t *const *ixs, int n_ix, gap_opt_t *opt, int n, const uint32_t *lens,
                              const uint64_t *offs, const uint8_t *codes, size_t codes_len, int32_t *n_aln,
                              uint32_t *flags, uint64_t *hit_off, uint32_t **hits, int32_t *splice_opt,
                              hsa_stats_t *stats)
{
    if (n_ix < 1 || n_ix > HSA_MAX_SLOTS) { hsa_gpu_set_error_text("1 to 16 device slots"); return HSA_E_ARG; }
    *hits = NULL;
    if (stats) memset(stats, 0, sizeof *stats);
    for (int r = 0; r < n; ++r)
        if (offs[r] > codes_len || lens[r] > codes_len - offs[r]) {
            char m[96];
            snprintf(m, sizeof m, "read %d: codes [%llu, +%u) past codes_len %zu", r, (unsigned long long)offs[r],
                     lens[r], codes_len);
            hsa_gpu_set_error_text(m);
            return HSA_E_ARG;
        }
    gap_opt_t local = *opt;                                 /* :254 */
    opt->mode &= ~BWA_MODE_GAPE;                            /* :261 through aux->opt */
    int max_len = 0, same_len = 1;
    for (int r = 0; r < n; ++r) {
        if ((int)lens[r] > max_len) max_len = (int)lens[r];
        if (lens[r] != lens[0]) same_len = 0;
    }
    if (opt->fnr > 0.0) local.max_diff = cal_maxdiff(max_len, BWA_AVG_ERR, opt->fnr);
    if (local.max_diff < local.max_gapo) local.max_gapo = local.max_diff;
    const int n_stacks = hsa_aln_score(&local, local.max_diff + 1, local.max_gapo + 1, local.max_gape + 1);
    /* every per-read max_diff of the call is <= local_opt.max_diff (bwtaln.c:264-267) */
    hsa_regime_t rg[2] = {hsa_regime_of(opt, n_stacks, local.max_diff), hsa_regime_of(&local, n_stacks, local.max_diff)};
    const int equivalent = same_len && memcmp(&rg[0], &rg[1], sizeof rg[0]) == 0;

    int8_t *kind = (int8_t *)malloc((size_t)n + 1);
    const double tm0 = hsa_now();
    readinfo_t *ri = (readinfo_t *)malloc(sizeof(readinfo_t) * ((size_t)n + 1));
    read_infos(codes, offs, lens, n, ri);
    const double tm1 = hsa_now();
    double tm_search = 0.0;
    int32_t *jmd = (int32_t *)malloc(sizeof(int32_t) * ((size_t)n + 1));
    int32_t *jsl = (int32_t *)malloc(sizeof(int32_t) * ((size_t)n + 1));
    hitbuf_t hb = {NULL, 0, 0};
    const optstate_t st0 = {opt->max_diff, opt->seed_len, local.max_diff, local.seed_len};
    optstate_t st = st0;
    int rc = 0, pos = 0, cur = 0, f_switch = -1;
    for (int r = 0; r < n; ++r) { n_aln[r] = 0; flags[r] = 0; hit_off[r] = 0; }

    while (pos < n && rc == 0) {
        if (cur == 0) {
            const int chunk = CHUNK0 * n_ix;                /* regime A is searched in chunks (Q2) */
            const int end = equivalent ? n : (pos + chunk < n ? pos + chunk : n);
            const optstate_t saved = st;
            for (int r = pos; r < end; ++r)
                kind[r] = (int8_t)plan_read(opt, 0, &st, ri + r, (int)lens[r], &jmd[r], &jsl[r]);
            const double ts = hsa_now();
            rc = search_range(ixs, n_ix, rg, pos, end, kind, jmd, jsl, 0, lens, offs, codes, codes_len, n_aln, flags,
                              hit_off, &hb, stats);
            tm_search += hsa_now() - ts;
            if (rc) break;
            int f = -1;
            for (int r = pos; r < end; ++r)
                if (kind[r] == K_JOB && (flags[r] & HSA_F_FALLBACK)) { f = r; break; }
            if (f >= 0) f_switch = f;
            if (f < 0 || equivalent) { pos = end; continue; }
            /* regime switch after read f: reads (f, end) are searched again in regime B */
            st = saved;
            for (int r = pos; r <= f; ++r)
                kind[r] = (int8_t)plan_read(opt, 0, &st, ri + r, (int)lens[r], &jmd[r], &jsl[r]);
            for (int r = f + 1; r < end; ++r) { n_aln[r] = 0; flags[r] = 0; hit_off[r] = 0; }
            cur = 1;
            pos = f + 1;
        } else {
            for (int r = pos; r < n; ++r)
                kind[r] = (int8_t)plan_read(opt, 1, &st, ri + r, (int)lens[r], &jmd[r], &jsl[r]);
            rc = search_range(ixs, n_ix, rg, pos, n, kind, jmd, jsl, 1, lens, offs, codes, codes_len, n_aln, flags,
                              hit_off, &hb, stats);
            pos = n;
        }
    }
    if (rc == 0) {
        /* replay the sequential prologue with the now-known switch point: final
         * option state, and the local_opt fields each fallback read's splice sees */
        optstate_t s = st0;
        int c = 0;
        for (int r = 0; r < n; ++r) {
            int32_t a, b;
            const int k = plan_read(opt, c, &s, ri + r, (int)lens[r], &a, &b);
            if (k == K_NFILTER) flags[r] = HSA_RF_NFILTER;
            else if (k == K_POLYAT) flags[r] = HSA_RF_POLYAT;
            if (splice_opt) { splice_opt[2 * r] = s.loc_max_diff; splice_opt[2 * r + 1] = s.loc_seed; }
            if (r == f_switch) c = 1;
        }
        opt->max_diff = s.opt_max_diff;
        opt->seed_len = s.opt_seed;
        *hits = hb.h ? hb.h : (uint32_t *)calloc(9, 4);
        if (getenv("HSA_VERBOSE"))
            fprintf(stderr, "[hsa] cal_sa_reg_gap of %d reads: filters %.1f ms, searches %.1f ms (kernels %.1f ms), "
                            "total %.1f ms\n", n, 1e3 * (tm1 - tm0), 1e3 * tm_search, stats ? stats->kernel_ms : -1.0,
                    1e3 * (hsa_now() - tm0));
    } else {
        free(hb.h);
    }
    free(kind); free(jmd); free(jsl); free(ri);
    return rc ? rc : (long)hb.n;
}

/* ------------------------------------------------------------------ reference ABI */

#define MAX_ATTACH 16
/* One attached Idx2BWT: its device index on every slot in use (slot k on device
 * k % hsa_device_count()).  The table is guarded by g_att_mu; an entry's slots are
 * only created, never replaced, while the Idx2BWT stays attached. */
static struct { const Idx2BWT *key; hsa_index_t *ix[HSA_MAX_SLOTS]; int n; } g_att[MAX_ATTACH];
static pthread_mutex_t g_att_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_slots = 0;                 /* 0: not chosen yet (HSA_GPU_DEVICES, else 1) */

static int slots_in_use(void)
{
    if (g_slots == 0) {
        const char *e = getenv("HSA_GPU_DEVICES");
        const int v = e ? atoi(e) : 1;
        g_slots = v >= 1 && v <= HSA_MAX_SLOTS ? v : 1;
    }
    return g_slots;
}

static int find_entry(const Idx2BWT *bi)
{
    for (int i = 0; i < MAX_ATTACH; ++i) if (g_att[i].key == bi) return i;
    return -1;
}

int hsa_gpu_set_devices(int n)
{
    if (n < 1 || n > HSA_MAX_SLOTS || hsa_device_count() < 1) return HSA_E_ARG;
    pthread_mutex_lock(&g_att_mu);
    g_slots = n;
    pthread_mutex_unlock(&g_att_mu);
    return 0;
}

/* Upload one slot's copy of the bidirectional BWT (and SA, blocks).  A slot on a device
 * that already holds one (slot >= device count) is a clone of that slot's index: the
 * same resident arrays, its own stream and scratch (hsa_index_clone). */
static int attach_slot(const Idx2BWT *bi, int slot, hsa_index_t *const *have, hsa_index_t **out)
{
    const BWT *f = bi->bwt, *r = bi->rev_bwt;
    const int nd = hsa_device_count();
    if (nd < 1) return HSA_E_NODEV;
    if (slot >= nd) return hsa_index_clone(have[slot % nd], out);
    hsa_index_t *ix = NULL;
    int rc = hsa_index_create(slot % nd, f->textLength, f->inverseSa0, f->cumulativeFreq, f->bwtCode,
                              r->textLength, r->inverseSa0, r->cumulativeFreq, r->bwtCode, &ix);
    /* SA -> position on the device needs the sampled SA (BWT.c:206-223) and blocks */
    if (rc == 0 && f->saValue && bi->hsp)
        rc = hsa_index_set_sa(ix, f->saValue, f->saValueSizeInWord, f->saInterval,
                              (const uint32_t *)bi->hsp->blockList, bi->hsp->numOfBlock);
    if (rc != 0 && ix) { hsa_index_free(ix); ix = NULL; }
    /* the splice kernel's motif scan and intron-end check read the packed reference as
     * the HSP holds it: (dnaLength + 15) / 16 + 1 words (DNALoadPacked,
     * TextConverter.c:704-707).  Only the splice kernel reads it: not uploaded with
     * HSA_SPLICE_DEVICE=0, and a failed upload (e.g. no HBM left) leaves the index without
     * it -- hsa_splice_device_launch then answers HSA_E_ARG and the host's path runs. */
    const char *sde = getenv("HSA_SPLICE_DEVICE");
    if (rc == 0 && ix && bi->hsp && bi->hsp->packedDNA && !(sde && atoi(sde) == 0)) {
        const int trc = hsa_index_set_text(ix, bi->hsp->packedDNA, ((uint64_t)bi->hsp->dnaLength + 15) / 16 + 1,
                                           bi->hsp->dnaLength);
        if (trc && getenv("HSA_VERBOSE"))
            fprintf(stderr, "[hsa] packed reference not uploaded (%s): the splice path runs on the host\n",
                    hsa_last_error());
    }
    *out = ix;
    return rc;
}

/* Two small searches on every slot at attach time, one without and one with gap opens:
 * the search kernels the first batches use are loaded before them (answers discarded). */
static void search_warm(const Idx2BWT *bi)
{
    int n_slots = 0;
    hsa_index_t *const *slots = hsa_gpu_slots_of(bi, &n_slots);
    uint8_t codes[2 * 100];
    for (int j = 0; j < 200; ++j) codes[j] = (uint8_t)((j * 5 + (j >> 4)) & 3);
    const uint32_t lens[2] = {100, 100};
    const uint64_t offs[2] = {0, 100};
    for (int gapo = 0; gapo < 2; ++gapo) {
        gap_opt_t o;
        memset(&o, 0, sizeof o);
        o.s_mm = 3; o.s_gapo = 11; o.s_gape = 4; o.max_diff = 4; o.max_gapo = gapo; o.max_gape = 6;   /* gap_init_opt */
        o.max_seed_diff = 2; o.seed_len = 32; o.max_entries = 2000000; o.max_top2 = 30; o.indel_end_skip = 5;
        o.max_del_occ = 10; o.fnr = -1.0f;
        int32_t n_aln[2], sp[4];
        uint32_t fl[2], *hits = NULL;
        uint64_t ho[2];
        if (hsa_cal_sa_reg_gap_multi(slots, n_slots, &o, 2, lens, offs, codes, sizeof codes, n_aln, fl, ho, &hits, sp,
                                     NULL) >= 0)
            hsa_free(hits);
    }
}

/* The device splice path once at attach, on synthetic reads (answers discarded), so that
 * the first batch does not pay for its kernels' first launches and first buffers.  By
 * default 4 096 reads: the prefetch pass's and the splice kernel's first launches, and
 * buffers for the few thousand fallback reads of a 100 000-read batch of unspliced reads
 * (the first call's device splice pass: 23 -> 13 ms with 64 reads).  HSA_SPLICE_WARM=1: a
 * batch the size of a host's batch of 150 bp reads (131 072 reads), so that the full-chip
 * buffers exist before the first batch too (their first allocation is ~0.2 s of the
 * first call); opt-in because those buffers stay allocated, which raised the footprint
 * enough to slow a second process sharing the GPU (the bench's end-to-end leg beside the
 * bench itself) from 0.26 s to 11 s per call.  HSA_SPLICE_WARM=0: none.  Non-fatal: a
 * failure is logged under HSA_VERBOSE. */
static void splice_device_warm(const Idx2BWT *bi)
{
    const char *sde = getenv("HSA_SPLICE_DEVICE"), *w = getenv("HSA_SPLICE_WARM");
    if ((sde && atoi(sde) == 0) || (w && atoi(w) == 0) || bwt_splice_match == NULL) return;
    int n_slots = 0;
    hsa_index_t *const *slots = hsa_gpu_slots_of(bi, &n_slots);
    if (n_slots < 1) return;
    enum { L_WARM = 150 };
    const int N_WARM = w && atoi(w) == 1 ? 131072 : 4096;
    uint32_t *lens = (uint32_t *)malloc(sizeof(uint32_t) * N_WARM);
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * N_WARM);
    int32_t *amd = (int32_t *)malloc(sizeof(int32_t) * N_WARM);
    uint8_t *codes = (uint8_t *)malloc((size_t)N_WARM * L_WARM);
    uint32_t *res = (uint32_t *)malloc(sizeof(uint32_t) * HSA_SP_RES_WORDS * (size_t)N_WARM);
    if (lens && offs && amd && codes && res) {
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (size_t j = 0; j < (size_t)N_WARM * L_WARM; ++j) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            codes[j] = (uint8_t)(x >> 62);
        }
        for (int k = 0; k < N_WARM; ++k) { lens[k] = L_WARM; offs[k] = (uint64_t)k * L_WARM; amd[k] = 4; }
        gap_opt_t o;                                  /* gap_init_opt, -n 4 -o 1 */
        memset(&o, 0, sizeof o);
        o.s_mm = 3; o.s_gapo = 11; o.s_gape = 4; o.max_diff = 4; o.max_gapo = 1; o.max_gape = 6;
        o.max_seed_diff = 2; o.seed_len = 32; o.max_entries = 2000000; o.max_top2 = 30; o.indel_end_skip = 5;
        o.max_del_occ = 10; o.fnr = -1.0f;
        const int n_stacks = hsa_aln_score(&o, o.max_diff + 1, o.max_gapo + 1, o.max_gape + 1);
        gap_opt_t so = o, ao = o;                     /* as dsp_job_run builds them */
        so.mode &= ~BWA_MODE_GAPE; so.max_gapo = 0; so.max_gape = 0; so.max_diff = o.max_seed_diff;
        ao.max_gape = 3;
        const hsa_regime_t srg = hsa_regime_of(&so, n_stacks, so.max_diff);
        const hsa_regime_t arg_ = hsa_regime_of(&ao, n_stacks, 4);
        hsa_regime_t erg = arg_;
        erg.mode = ao.mode & (BWA_MODE_GAPE | BWA_MODE_LOGGAP | BWA_MODE_NONSTOP);
        hsa_splice_pf_t pf;
        hsa_splice_stats_t st;
        const double t0 = hsa_now();
        int rc = 0;
        hsa_gpu_lock();
        for (int k = 0; k < n_slots && !rc; ++k)     /* each device loads the kernels */
            rc = hsa_splice_match_batch(slots[k], &srg, &arg_, &erg, N_WARM, lens, offs, codes,
                                        (size_t)N_WARM * L_WARM, amd, &pf, res, &st);
        hsa_gpu_unlock();
        if (getenv("HSA_VERBOSE"))
            fprintf(stderr, "[hsa] splice path warm-up: %d reads, %.3f s%s%s\n", N_WARM, hsa_now() - t0,
                    rc ? ", failed: " : "", rc ? hsa_last_error() : "");
    }
    free(lens); free(offs); free(amd); free(codes); free(res);
}

/* Upload the bidirectional BWT of a loaded Idx2BWT once per slot in use (hook after
 * BWTLoad2BWT); slots added later by hsa_gpu_set_devices are attached on first use. */
int hsa_gpu_attach(const Idx2BWT *bi)
{
    pthread_mutex_lock(&g_att_mu);
    const int want = slots_in_use();
    int e = find_entry(bi);
    if (e < 0) {
        for (int i = 0; i < MAX_ATTACH; ++i) if (!g_att[i].key) { e = i; break; }
        if (e < 0) { pthread_mutex_unlock(&g_att_mu); return HSA_E_ARG; }
        g_att[e].key = bi;
        g_att[e].n = 0;
    }
    int rc = 0;
    while (g_att[e].n < want && rc == 0) {
        hsa_index_t *ix = NULL;
        rc = attach_slot(bi, g_att[e].n, g_att[e].ix, &ix);
        if (rc == 0) g_att[e].ix[g_att[e].n++] = ix;
    }
    if (g_att[e].n == 0) g_att[e].key = NULL;
    pthread_mutex_unlock(&g_att_mu);
    /* the splice path's host and device resources, made before the first batch needs them */
    if (rc == 0) {
        /* Every batch hands the host ~100 000 calloc'd hit arrays (bwt_match_gap's contract,
         * bwtgap.c:137-138) that the host frees before the next batch (bwaseqio.c:244).
         * glibc returns the freed pages to the kernel by default, so each batch re-faults
         * them (~20 ms per 100 000 reads); keeping them in the heap makes the next batch's
         * arrays reuse them.  It changes the whole process's malloc, so it is opt-in:
         * HSA_MALLOC_TUNE=1.  Results do not depend on it. */
        const char *mt = getenv("HSA_MALLOC_TUNE");
        static int tuned = 0;
        if (!tuned && mt && atoi(mt) != 0) {
            mallopt(M_TRIM_THRESHOLD, 1 << 30);
            mallopt(M_MMAP_THRESHOLD, 64 << 20);
            tuned = 1;
            /* and the heap those arrays take for a 100 000-read batch, made now: its pages
             * faulted in once, here, and kept */
            enum { N_WARM = 120000 };
            void **w = (void **)malloc(sizeof(void *) * N_WARM);
            if (w) {
                for (int i = 0; i < N_WARM; ++i) w[i] = calloc(10, sizeof(bwt_aln1_t));
                for (int i = N_WARM - 1; i >= 0; --i) free(w[i]);
                free(w);
            }
        }
        search_warm(bi);
        if (hsa_splice_warm && hsa_splice_extend_active && hsa_splice_extend_active()) hsa_splice_warm(4096);
        if (hsa_splice_prefetch_warm && hsa_splice_prefetch_active && hsa_splice_prefetch_active())
            hsa_splice_prefetch_warm(bi);
        splice_device_warm(bi);
    }
    return rc;
}

void hsa_gpu_detach(const Idx2BWT *bi)
{
    pthread_mutex_lock(&g_att_mu);
    const int e = find_entry(bi);
    if (e >= 0) {
        for (int k = g_att[e].n - 1; k >= 0; --k) hsa_index_free(g_att[e].ix[k]);   /* clones first */
        memset(&g_att[e], 0, sizeof g_att[e]);
    }
    pthread_mutex_unlock(&g_att_mu);
}

/* The device indexes of a loaded Idx2BWT on the slots in use, attached on first use
 * (bwtaln_gpu.h); *n receives the slot count. */
hsa_index_t *const *hsa_gpu_slots_of(const Idx2BWT *bi, int *n)
{
    pthread_mutex_lock(&g_att_mu);
    const int want = slots_in_use();
    const int e = find_entry(bi);
    const int ok = e >= 0 && g_att[e].n >= want;
    pthread_mutex_unlock(&g_att_mu);
    if (!ok) {
        long rc = hsa_gpu_attach(bi);
        if (rc) hsa_gpu_fatal("hsa_gpu_attach", rc);
    }
    pthread_mutex_lock(&g_att_mu);
    const int e2 = find_entry(bi);
    hsa_index_t *const *ix = g_att[e2].ix;
    *n = want;
    pthread_mutex_unlock(&g_att_mu);
    return ix;
}

/* The device index of slot 0 (the splice path's direct bwt_match_gap calls). */
hsa_index_t *hsa_gpu_index_of(const Idx2BWT *bi)
{
    int n = 0;
    return hsa_gpu_slots_of(bi, &n)[0];
}

/* gap_init_stack layout (bwtgap.c:13-27), for the host's bwt_splice_match */
static gap_stack_t *ref_stack_new(int n_stacks)
{
    gap_stack_t *s = (gap_stack_t *)calloc(1, sizeof(gap_stack_t));
    s->n_stacks = n_stacks;
    s->stacks = (gap_stack1_t *)calloc(n_stacks, sizeof(gap_stack1_t));
    for (int i = 0; i < n_stacks; ++i) {
        s->stacks[i].m_entries = 4;
        s->stacks[i].stack = (gap_entry_t *)calloc(4, sizeof(gap_entry_t));
    }
    return s;
}

static void ref_stack_free(gap_stack_t *s)
{
    for (int i = 0; i < s->n_stacks; ++i) free(s->stacks[i].stack);
    free(s->stacks);
    free(s);
}

static pthread_mutex_t g_call_mu;
static pthread_once_t g_call_once = PTHREAD_ONCE_INIT;

static void call_mu_init(void)
{
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_settype(&a, PTHREAD_MUTEX_RECURSIVE);
    pthread_mutex_init(&g_call_mu, &a);
    pthread_mutexattr_destroy(&a);
}

void hsa_gpu_lock(void)
{
    pthread_once(&g_call_once, call_mu_init);
    pthread_mutex_lock(&g_call_mu);
}

void hsa_gpu_unlock(void) { pthread_mutex_unlock(&g_call_mu); }

double hsa_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

void hsa_gpu_fatal(const char *what, long rc)
{
    /* the reference's convention for unrecoverable errors: message + exit(1) */
    fprintf(stderr, "[bwa_cal_sa_reg_gap] %s failed (%ld): %s\n", what, rc, hsa_last_error());
    exit(1);
}

/* One drop-in call at a time: the batch's splice prefetch table (bwtgap_gpu.c) and the
 * splice runner's coroutine pool (bwtext_gpu.c) are process-wide, so concurrent callers
 * (the reference has none: its thread loop is commented out, bwtaln.c:483-506) are
 * serialised here rather than sharing them. */
static pthread_mutex_t g_batch_mu = PTHREAD_MUTEX_INITIALIZER;

/* The splice kernel's guard: the kernel restates the reference's bwt_splice_match
 * (bwtgap.c:748-1332) and the drop-in uses it in place of the host's function, which is
 * right only while the host's function is the reference's (its splice-site record,
 * bwt_array_insert / bwt_find_split_pos_by_record, returns at entry: bwt_array.c:34,
 * :77).  So on the first batch with device answers the host's own function also runs
 * for the first SP_GUARD answered reads; any difference turns the device path off for
 * the rest of the process (logged once).  0 unchecked, 1 checked, -1 off.  Guarded by
 * g_batch_mu. */
#define SP_GUARD 64
static int g_sp_guard = 0;

/* a device answer (HSA_SP_RES_WORDS words: status, n_aln, res_aln[0..1]) as the host's
 * bwt_splice_match would leave it: a calloc(2) result array (bwtgap.c:854) */
static void put_device_answer(bwa_seq_t *p, const uint32_t *o)
{
    p->n_aln = (int)o[1];
    if (o[1] == 0) { p->aln = NULL; return; }
    p->aln = (bwt_aln1_t *)calloc(2, sizeof(bwt_aln1_t));
    memcpy(p->aln, o + 2, 2 * sizeof(bwt_aln1_t));
}

/* What the host's splice path of one batch needs. */
typedef struct {
    const Idx2BWT *bi;
    struct bwt_array_t *arr;
    bwa_seq_t *seqs;
    const uint64_t *offs;
    size_t tot;
    int max_len;
    const gap_opt_t *local;
    const int32_t *sp;
    int n_stacks;
    int have_splice;
    int pf_ok;
} host_ctx_t;

/* The host's bwt_splice_match for reads hr[0..n) (ascending; read q of them is number q
 * of the batch's prefetch table when `prefetched`): all of them at once as coroutines
 * whose seed extensions run batched on the GPU, when the host calls our bwt_extend_*
 * (bwtext_gpu.c); else one read at a time, as the reference. */
static void run_host_reads(const host_ctx_t *c, const int *hr, int n, int prefetched)
{
    const int batched = c->have_splice && hsa_splice_run && hsa_splice_extend_active && hsa_splice_extend_active();
    hsa_splice_read_t *sr = NULL;
    int *sr_idx = NULL, n_sr = 0;
    bwt_aux_t aux;
    memset(&aux, 0, sizeof aux);
    if (batched) {
        sr = (hsa_splice_read_t *)malloc(sizeof(hsa_splice_read_t) * ((size_t)n + 1));
        sr_idx = (int *)malloc(sizeof(int) * ((size_t)n + 1));
    }
    for (int q = 0; q < n; ++q) {
        const int i = hr[q];
        bwa_seq_t *p = c->seqs + i;
        gap_opt_t lo = *c->local;                               /* aux->opt = &local_opt (:363) */
        lo.max_diff = c->sp[2 * i];
        lo.seed_len = c->sp[2 * i + 1];
        if (batched) {
            sr[n_sr].seq = p->seq; sr[n_sr].len = (int)p->len; sr[n_sr].opt = lo;
            sr_idx[n_sr++] = i;
            continue;
        }
        if (!aux.stack) {
            aux.bi_bwt = (Idx2BWT *)c->bi;
            aux.arr = c->arr;
            aux.max_len = c->max_len;
            aux.width_back = (bwt_width_t *)calloc(c->max_len + 1, sizeof(bwt_width_t));
            aux.width_fore = (bwt_width_t *)calloc(c->max_len + 1, sizeof(bwt_width_t));
            aux.width_seed = (bwt_width_t *)calloc(c->max_len + 1, sizeof(bwt_width_t));
            aux.rc_seq = (ubyte_t *)calloc(c->max_len + 1, 1);
            aux.stack = ref_stack_new(c->n_stacks);
        }
        aux.opt = &lo;
        aux.seq = p->seq;
        aux.len = (int)p->len;
        aux.strand = 0;
        memset(aux.rc_seq, 0, (size_t)c->max_len);
        for (int j = 0; j < (int)p->len; ++j) {
            ubyte_t ch = p->seq[p->len - 1 - j];
            aux.rc_seq[j] = ch < 4 ? (ubyte_t)(3 - ch) : ch;
        }
        int na = 0;
        if (hsa_splice_set_read) hsa_splice_set_read(prefetched ? q : -1);
        p->aln = bwt_splice_match(&aux, &na);
        if (hsa_splice_set_read) hsa_splice_set_read(-1);
        p->n_aln = na;
        if (na == 0) { free(p->aln); p->aln = NULL; }
    }
    if (n_sr > 0) {
        bwt_aln1_t **so = (bwt_aln1_t **)malloc(sizeof(bwt_aln1_t *) * (size_t)n_sr);
        int *sn = (int *)malloc(sizeof(int) * (size_t)n_sr);
        const long launches = hsa_splice_run(c->bi, c->arr, c->max_len, c->n_stacks, n_sr, sr, so, sn);
        for (int k = 0; k < n_sr; ++k) {
            bwa_seq_t *p = c->seqs + sr_idx[k];
            p->aln = so[k];
            p->n_aln = sn[k];
            if (sn[k] == 0) { free(p->aln); p->aln = NULL; }
        }
        if (getenv("HSA_VERBOSE"))
            fprintf(stderr, "[hsa] splice path: %d reads as coroutines, seed extensions in %ld GPU launches\n", n_sr,
                    launches);
        free(so); free(sn);
    }
    free(sr); free(sr_idx);
    if (aux.stack) {
        free(aux.width_back); free(aux.width_fore); free(aux.width_seed); free(aux.rc_seq);
        ref_stack_free(aux.stack);
    }
    if (prefetched) {
        if (getenv("HSA_VERBOSE") && hsa_splice_memo_stats) {
            uint64_t mh = 0, mm = 0, wh = 0, wm = 0, sh = 0, sm = 0;
            hsa_splice_memo_stats(&mh, &mm);
            if (hsa_splice_table_stats) hsa_splice_table_stats(&wh, &wm, &sh, &sm);
            fprintf(stderr, "[hsa] splice prefetch: %llu bwt_match_gap calls answered from the batch, %llu run alone; "
                            "%llu bwt_cal_width calls from the batch, %llu alone; %llu SA lookups from the batch, %llu "
                            "not\n", (unsigned long long)mh, (unsigned long long)mm, (unsigned long long)wh,
                    (unsigned long long)wm, (unsigned long long)sh, (unsigned long long)sm);
        }
        hsa_splice_memo_clear();
    }
    /* the runner's rounds add their lookups to the SA table: clear it after every batch
     * that ran the coroutine runner, so it never outgrows a batch */
    if (n_sr > 0 && hsa_splice_sa_clear) {
        if (getenv("HSA_VERBOSE") && hsa_splice_sa_stats) {
            uint64_t sh = 0, sm = 0;
            hsa_splice_sa_stats(&sh, &sm);
            fprintf(stderr, "[hsa] splice SA -> position: %llu lookups answered from the batch, %llu in the runner's "
                            "rounds\n", (unsigned long long)sh, (unsigned long long)sm);
        }
        hsa_splice_sa_clear();
    }
}

static void cal_sa_reg_gap_locked(const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, const gap_opt_t *copt,
                                  struct bwt_array_t *arr);

void bwa_cal_sa_reg_gap(int tid, const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, const gap_opt_t *copt,
                        struct bwt_array_t *arr)
{
    (void)tid;
    pthread_mutex_lock(&g_batch_mu);
    cal_sa_reg_gap_locked(bi_bwt, n_seqs, seqs, copt, arr);
    pthread_mutex_unlock(&g_batch_mu);
}

static void cal_sa_reg_gap_locked(const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, const gap_opt_t *copt,
                                  struct bwt_array_t *arr)
{
    gap_opt_t *opt = (gap_opt_t *)copt;     /* mutated, as the reference does through aux->opt */
    int n_slots = 1;
    hsa_index_t *const *slots = hsa_gpu_slots_of(bi_bwt, &n_slots);
    uint32_t *lens = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)n_seqs + 1));
    uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n_seqs + 1));
    size_t tot = 0;
    int max_len = 0;
    for (int i = 0; i < n_seqs; ++i) {
        lens[i] = seqs[i].len; offs[i] = tot; tot += seqs[i].len;
        if ((int)seqs[i].len > max_len) max_len = (int)seqs[i].len;
    }
    uint8_t *codes = (uint8_t *)malloc(tot + 1);
    for (int i = 0; i < n_seqs; ++i) memcpy(codes + offs[i], seqs[i].seq, seqs[i].len);
    int32_t *n_aln = (int32_t *)malloc(sizeof(int32_t) * ((size_t)n_seqs + 1));
    uint32_t *flags = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)n_seqs + 1));
    uint64_t *hoff = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n_seqs + 1));
    int32_t *sp = (int32_t *)malloc(sizeof(int32_t) * 2 * ((size_t)n_seqs + 1));
    gap_opt_t local = *opt;                 /* local_opt as of :254, before the call mutates *opt */
    uint32_t *hits = NULL;
    const double t0 = hsa_now();
    long nh = hsa_cal_sa_reg_gap_multi(slots, n_slots, opt, n_seqs, lens, offs, codes, tot, n_aln, flags, hoff, &hits, sp,
                                       NULL);
    if (nh < 0) hsa_gpu_fatal("GPU search", nh);
    if (opt->fnr > 0.0) local.max_diff = cal_maxdiff(max_len, BWA_AVG_ERR, opt->fnr);
    if (local.max_diff < local.max_gapo) local.max_gapo = local.max_diff;

    const int have_splice = bwt_splice_match != NULL;
    const int n_stacks = hsa_aln_score(&local, local.max_diff + 1, local.max_gapo + 1, local.max_gape + 1);
    /* the reads that go to bwt_splice_match (bwtaln.c:362-369), in order */
    int *fb = (int *)malloc(sizeof(int) * ((size_t)n_seqs + 1));
    int nf = 0;
    for (int i = 0; i < n_seqs; ++i)
        if (!(flags[i] & (HSA_RF_NFILTER | HSA_RF_POLYAT)) && n_aln[i] == 0 && (flags[i] & HSA_F_FALLBACK) && have_splice)
            fb[nf++] = i;
    const double t1 = hsa_now();
    /* bwt_splice_match of every fallback read on the device (hsa_splice_match_batch: the
     * prefetch pass and the splice kernel, hsa_splice.hip), on helper threads -- the reads
     * split into contiguous parts, one per device slot -- while this thread writes the
     * per-read output arrays (so that they come from the host thread's own heap arena,
     * where the host frees them).  HSA_SPLICE_DEVICE=0, or a host whose bwt_splice_match
     * answers differently (the guard below): the host's bwt_splice_match for all of them. */
    const char *sde = getenv("HSA_SPLICE_DEVICE");
    const int want_dev = !sde || atoi(sde) != 0;
    int dev = want_dev && g_sp_guard >= 0 && nf > 0 && n_stacks <= HSA_SP_MAX_STACKS;
    for (int k = 0; dev && k < nf; ++k)
        if (seqs[fb[k]].len < 3 || seqs[fb[k]].len > 3 * 1021) dev = 0;   /* the prefetch's read lengths */
    const int n_dj = dev ? (n_slots < nf ? n_slots : nf) : 0;
    dsp_job_t dj[HSA_MAX_SLOTS];
    pthread_t dth[HSA_MAX_SLOTS];
    int dev_async[HSA_MAX_SLOTS] = {0};
    uint32_t *dres = dev ? (uint32_t *)malloc(sizeof(uint32_t) * HSA_SP_RES_WORDS * (size_t)nf) : NULL;
    for (int k = 0; k < n_dj; ++k) {
        const int j0 = (int)((long)nf * k / n_dj), j1 = (int)((long)nf * (k + 1) / n_dj);
        memset(&dj[k], 0, sizeof dj[k]);
        dj[k].ix = slots[k]; dj[k].n = j1 - j0; dj[k].fb = fb + j0; dj[k].seqs = seqs; dj[k].sp = sp;
        dj[k].local = local; dj[k].n_stacks = n_stacks; dj[k].res = dres + (size_t)HSA_SP_RES_WORDS * j0;
        dj[k].lock = k == 0;
        dev_async[k] = pthread_create(&dth[k], NULL, dsp_job_run, &dj[k]) == 0;
        if (!dev_async[k]) dsp_job_run(&dj[k]);
    }
    /* the splice path's widths, seed and anchor searches and SA lookups of the host's reads
     * in one device pass (hsa_splice_prefetch, bwtgap_gpu.c), when the host's
     * bwt_splice_match calls our bwt_match_gap.  HSA_SPLICE_PREFETCH=0: no table, every
     * splice-path call goes to the GPU on its own (tests: misses from several runner
     * threads at once) */
    const char *pfe = getenv("HSA_SPLICE_PREFETCH");
    const int want_pf = !pfe || atoi(pfe) != 0;
    const host_ctx_t hc = {bi_bwt, arr, seqs, offs, tot, max_len, &local, sp, n_stacks, have_splice,
                           want_pf && have_splice && hsa_splice_prefetch_active && hsa_splice_prefetch_active()};
    /* the reads the host's bwt_splice_match runs: all fallback reads, or those the device
     * did not answer (+ the guard's); hr[] in order, numbered in the prefetch table by
     * their rank in hr */
    int *hr = fb, nh_r = nf;
    pf_job_t pj;
    memset(&pj, 0, sizeof pj);
    pthread_t pth;
    int pf_async = 0, prefetched = 0;
    double t_pf = 0.0;
    if (!dev && hc.pf_ok && nh_r > 0) {      /* beside the per-read outputs */
        pf_job_init(&pj, bi_bwt, arr, seqs, offs, tot, max_len, hr, nh_r, &local, sp, n_stacks);
        pf_async = pthread_create(&pth, NULL, pf_job_run, &pj) == 0;
        if (!pf_async) pf_job_run(&pj);
        prefetched = 1;
    }
    const double to = hsa_now();
    write_outputs(seqs, n_seqs, n_aln, flags, hoff, hits);
    const double t_out = hsa_now() - to;
    if (pf_async) pthread_join(pth, NULL);
    for (int k = 0; k < n_dj; ++k) if (dev_async[k]) pthread_join(dth[k], NULL);
    const double t_join = hsa_now() - to - t_out;
    int n_dev = 0, n_spl = 0, n_guard = 0, *gd = NULL;       /* gd: the guard's reads, their numbers in fb */
    if (dev) {
        int rc = 0;
        hsa_splice_stats_t st;
        memset(&st, 0, sizeof st);
        double dsecs = 0.0;
        for (int k = 0; k < n_dj; ++k) {
            if (dj[k].rc && !rc) rc = dj[k].rc;
            st.extensions += dj[k].st.extensions; st.pops += dj[k].st.pops; st.sa_lookups += dj[k].st.sa_lookups;
            st.kernel_ms += dj[k].st.kernel_ms;
            if (dj[k].secs > dsecs) dsecs = dj[k].secs;
        }
        if (rc == HSA_E_ARG || rc == HSA_E_MEM) {
            /* not on this index / these options, or no device memory for its buffers (another
             * process may hold the HBM): the host's path, as with HSA_SPLICE_DEVICE=0 */
            if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] splice kernel not used: %s\n", hsa_last_error());
        } else if (rc) {
            hsa_gpu_fatal("GPU splice path", rc);
        } else {
            /* the device's answers; the reads it did not answer go to the host's path.  On the
             * process's first batch with device answers, the host also runs its own
             * bwt_splice_match for the first SP_GUARD answered reads (the guard) */
            hr = (int *)malloc(sizeof(int) * ((size_t)nf + 1));
            gd = (int *)malloc(sizeof(int) * SP_GUARD);
            nh_r = 0;
            for (int k = 0; k < nf; ++k) {
                const uint32_t *o = dres + (size_t)HSA_SP_RES_WORDS * k;
                if (o[0] != HSA_SP_OK) { hr[nh_r++] = fb[k]; continue; }
                if (g_sp_guard == 0 && n_guard < SP_GUARD) { gd[n_guard++] = k; hr[nh_r++] = fb[k]; continue; }
                put_device_answer(seqs + fb[k], o);
                ++n_dev;
                n_spl += o[1] > 0;
            }
            if (getenv("HSA_VERBOSE"))
                fprintf(stderr, "[hsa] splice kernel: %d reads, %d spliced, %d to the host's path (%d of them the "
                                "guard's), %d slot(s); %llu extensions, %llu pops, %llu SA lookups, %.1f ms of kernel "
                                "(%.3f s with the prefetch pass)\n", nf, n_spl, nh_r, n_guard, n_dj, (unsigned long long)st.extensions, (unsigned long long)st.pops,
                        (unsigned long long)st.sa_lookups, st.kernel_ms, dsecs);
        }
        t_pf = dsecs;
    }
    if (dev && hc.pf_ok && nh_r > 0) {          /* the host's reads' own prefetch (all of them when the
                                                 * device path gave way) */
        pf_job_init(&pj, bi_bwt, arr, seqs, offs, tot, max_len, hr, nh_r, &local, sp, n_stacks);
        pf_job_run(&pj);
        prefetched = 1;
    }
    if (prefetched) {
        t_pf += pj.secs;
        pf_job_free(&pj);
    }
    const double t2 = hsa_now();
    run_host_reads(&hc, hr, nh_r, prefetched);
    if (n_guard > 0) {
        /* the guard: the host's answers for these reads against the device's */
        int bad = -1;
        for (int g = 0; g < n_guard && bad < 0; ++g) {
            const uint32_t *o = dres + (size_t)HSA_SP_RES_WORDS * gd[g];
            const bwa_seq_t *p = seqs + fb[gd[g]];
            if (p->n_aln != (int)o[1] || (o[1] > 0 && memcmp(p->aln, o + 2, sizeof(bwt_aln1_t) * o[1]) != 0)) bad = g;
        }
        if (bad < 0) g_sp_guard = 1;
        else {
            g_sp_guard = -1;
            fprintf(stderr, "[hsa] the host's bwt_splice_match answers read %d of this batch differently from the "
                            "splice kernel (bwtgap.c:748): the host's function runs every fallback read from now on\n",
                    fb[gd[bad]]);
            /* this batch's device answers go too: the host runs those reads as well */
            int n2 = 0;
            int *h2 = (int *)malloc(sizeof(int) * ((size_t)nf + 1));
            for (int k = 0, g = 0; k < nf; ++k) {
                if (g < n_guard && gd[g] == k) { ++g; continue; }
                if (dres[(size_t)HSA_SP_RES_WORDS * k] != HSA_SP_OK) continue;
                bwa_seq_t *p = seqs + fb[k];
                free(p->aln);
                p->aln = NULL; p->n_aln = 0;
                h2[n2++] = fb[k];
            }
            n_dev = 0;
            int pf2 = 0;
            if (hc.pf_ok && n2 > 0) {
                pf_job_init(&pj, bi_bwt, arr, seqs, offs, tot, max_len, h2, n2, &local, sp, n_stacks);
                pf_job_run(&pj);
                t_pf += pj.secs;
                pf_job_free(&pj);
                pf2 = 1;
            }
            run_host_reads(&hc, h2, n2, pf2);
            free(h2);
        }
    }
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] batch of %d reads: search %.3f s, splice prefetch %.3f s, splice path %.3f s "
                        "(%d fallback reads, %d on the device; per-read outputs %.1f ms%s, %.1f ms waited for)\n",
                n_seqs, t1 - t0, t_pf, hsa_now() - t2 + (t2 - t1 - t_pf), nf, n_dev, 1e3 * t_out,
                (prefetched || dev) ? " beside the device pass" : "", 1e3 * t_join);
    free(dres);
    free(gd);
    if (hr != fb) free(hr);
    free(fb);
    hsa_free(hits);
    free(lens); free(offs); free(codes); free(n_aln); free(flags); free(hoff); free(sp);
}
