/*
 * bwtext_gpu.c -- the splice path's seed extensions on the GPU, and the batched runner
 * of the host's splice path that feeds them.
 *
 * bwt_extend_backward / bwt_extend_foreward (bwtgap.c:640-663, declared bwtgap.h) are
 * what bwt_splice_match (bwtgap.c:748) calls to grow a mapped seed across the read:
 * bwt_backtracing_search (:346-511), the splice path's costliest host step once its
 * bwt_match_gap calls run on the GPU.  Each call depends on the previous one's result,
 * so one read's calls cannot be batched; the calls of many reads can.  So the drop-in
 * bwa_cal_sa_reg_gap runs bwt_splice_match -- the host's own code, unchanged -- for
 * every fallback read of a batch as a coroutine (ucontext, one stack each, one host
 * thread): a coroutine that calls bwt_extend_* parks its call and yields; when every
 * running coroutine is parked or done, one hsa_extend_batch launch answers all parked
 * calls and they resume.  bwt_splice_match is a function of its read alone (its
 * splice-site record, bwt_array_t, is inert: bwt_array_insert and
 * bwt_find_split_pos_by_record return at their first line, bwt_array.c:34, :77), so
 * the reads' order does not change any result.
 *
 * The same object answers the splice path's bwt_cal_width calls (bwtaln.c:73, called at
 * bwtgap.c:807, :867-868, :871-872, :915) from the per-read table the drop-in fills on
 * the GPU ahead of the splice path (hsa_splice_prefetch, bwtgap_gpu.c): every width array
 * those calls can ask for, per fallback read and strand.
 *
 * Its own object: a host opts in by linking bwtext_gpu.o and weakening its own
 * bwt_extend_backward / bwt_extend_foreward / bwt_cal_width.
 */
#define _GNU_SOURCE
/* coroutine switches _longjmp between stacks, which the fortified longjmp refuses */
#undef _FORTIFY_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <setjmp.h>
#include <sys/mman.h>
#include <ucontext.h>

#include "../../include/hsa_bwtaln.h"
#include "bwtaln_gpu.h"

#define CO_STACK (512u << 10)     /* C stack per coroutine (the host's splice code + ours) */
#define CO_GUARD 4096u            /* PROT_NONE page under each coroutine stack */
#define CO_MAX 16384              /* coroutines alive at once (= extension slots) */
#define SLICE_POPS 256u           /* pops per call per launch (hsa_extend_sliced) */

/* One parked extension call. */
typedef struct {
    int dir, len, max_pos;
    hsa_regime_t rg;
    int lo, n;
    uint8_t *seq;                 /* window copies (in buf when owned == 0) */
    int32_t *bid;
    int owned;                    /* seq / bid malloc'd by fill_req */
    uint8_t *buf;                 /* the coroutine's window buffer, or NULL */
    size_t buf_cap;
    bwt_aln1_t *aln;              /* the caller's, updated on resume */
    int *max_pos_io;
    int ret;
    int started;                  /* sliced: submitted before, its state is in its slot */
    int kind;                     /* 0 an extension, 1 an SA -> position lookup */
    uint32_t sa;                  /* kind 1: the SA index, and where its answer goes */
    unsigned int *sid_p, *ori_p, *occ_p;
} ext_req_t;

typedef struct {
    ucontext_t uc;                /* the coroutine's first entry (makecontext) */
    jmp_buf jb;                   /* where it parked (switches use _setjmp/_longjmp: no
                                     signal-mask system calls, unlike swapcontext) */
    int entered;
    void *stack;
    int read;                     /* index into the run's reads, -1 idle */
    int state;                    /* 0 runnable, 1 parked, 2 done */
    bwt_aux_t aux;
    gap_opt_t opt;
    int len;                      /* the read's length */
    bwt_aln1_t *result;
    int n_aln;
    ext_req_t req;
} co_t;

static __thread co_t *tl_co;          /* the running coroutine, or NULL outside the runner */
static __thread jmp_buf *tl_sched;    /* the runner's resume point */

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* The window of read positions a call reads (include/hsa_gpu.h, hsa_ext_job_t):
 * backward [min(start - len, max_pos), max(start, max_pos + 1)], forward
 * [min(end, max_pos - 1), max(end + len, max_pos)]; empty for a negative len without
 * NONSTOP (the seed entry's score field is 2047 then: the search stops at its first
 * pop).  Returns 0, or -1 when the reference's search would read undefined memory. */
static int call_window(const bwt_aux_t *aux, const bwt_aln1_t *aln, int dir, int max_pos, int read_len, int *lo,
                       int *n)
{
    const int len = aux->len;
    if (len < 0 && !(aux->opt->mode & BWA_MODE_NONSTOP)) { *lo = 0; *n = 0; return 0; }
    int l, h;
    if (dir) { l = imin(aln->start - len, max_pos); h = imax(aln->start, max_pos + 1); }
    else { l = imin(aln->end, max_pos - 1); h = imax(aln->end + len, max_pos); }
    if (len < 0 || l < 0 || (read_len >= 0 && h > read_len)) return -1;
    *lo = l;
    *n = h - l + 1;
    return 0;
}

static void fill_req(ext_req_t *q, bwt_aux_t *aux, bwt_aln1_t *aln, int *max_pos, int dir, int read_len)
{
    q->dir = dir;
    q->len = aux->len;
    q->max_pos = *max_pos;
    q->rg = hsa_regime_of(aux->opt, aux->stack->n_stacks, aux->opt->max_diff);
    q->rg.mode = aux->opt->mode & (BWA_MODE_GAPE | BWA_MODE_LOGGAP | BWA_MODE_NONSTOP);   /* as the search reads it */
    q->rg.max_gapo = aux->opt->max_gapo;
    q->rg.max_gape = aux->opt->max_gape;
    if (call_window(aux, aln, dir, *max_pos, read_len, &q->lo, &q->n)) {
        fprintf(stderr, "[bwt_extend_%s] extension of %d positions from [%d, %d] toward %d reads outside the read "
                        "(undefined in the reference)\n", dir ? "backward" : "foreward", aux->len, aln->start, aln->end,
                *max_pos);
        exit(1);
    }
    const ubyte_t *seq = aux->strand == 0 ? aux->seq : aux->rc_seq;
    const bwt_width_t *w = dir ? aux->width_back : aux->width_fore;
    /* the sequence is read only at [start - len, start - 1] / [end + 1, end + len] */
    const int s0 = dir ? aln->start - aux->len : aln->end + 1, s1 = dir ? aln->start - 1 : aln->end + aux->len;
    const size_t need = 4 * ((size_t)q->n + 1) + (size_t)q->n + 1;
    if (q->buf && need <= q->buf_cap) {
        q->bid = (int32_t *)q->buf;
        q->seq = q->buf + 4 * ((size_t)q->n + 1);
        q->owned = 0;
    } else {
        q->seq = (uint8_t *)malloc((size_t)q->n + 1);
        q->bid = (int32_t *)malloc(sizeof(int32_t) * ((size_t)q->n + 1));
        q->owned = 1;
    }
    for (int p = 0; p < q->n; ++p) {
        const int pos = q->lo + p;
        q->seq[p] = pos >= s0 && pos <= s1 ? seq[pos] : 4;
        q->bid[p] = w[pos].bid;
    }
    q->aln = aln;
    q->max_pos_io = max_pos;
}

/* Answer parked calls q[0..n) in one batch. */
static void run_reqs(hsa_index_t *ix, ext_req_t *const *q, int n)
{
    if (n <= 0) return;
    hsa_regime_t *rg = (hsa_regime_t *)calloc((size_t)n, sizeof(hsa_regime_t));
    hsa_ext_job_t *jobs = (hsa_ext_job_t *)calloc((size_t)n, sizeof(hsa_ext_job_t));
    size_t tot = 0;
    for (int j = 0; j < n; ++j) tot += (size_t)q[j]->n;
    uint8_t *codes = (uint8_t *)calloc(tot + 1, 1);
    int32_t *bids = (int32_t *)calloc(tot + 1, sizeof(int32_t));
    int nr = 0;
    size_t off = 0;
    for (int j = 0; j < n; ++j) {
        int r = 0;
        while (r < nr && memcmp(&rg[r], &q[j]->rg, sizeof(hsa_regime_t))) ++r;
        if (r == nr) rg[nr++] = q[j]->rg;
        hsa_ext_job_t *J = jobs + j;
        J->dir = q[j]->dir; J->len = q[j]->len; J->max_pos = q[j]->max_pos; J->regime = r;
        J->lo = q[j]->lo; J->n = q[j]->n; J->off = off;
        memcpy(J->aln, q[j]->aln, sizeof(bwt_aln1_t));
        memcpy(codes + off, q[j]->seq, (size_t)q[j]->n);
        memcpy(bids + off, q[j]->bid, sizeof(int32_t) * (size_t)q[j]->n);
        off += (size_t)q[j]->n;
    }
    int32_t *ret = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t *mp = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    uint32_t *aln = (uint32_t *)malloc(sizeof(bwt_aln1_t) * (size_t)n);
    hsa_gpu_lock();
    int rc = hsa_extend_batch(ix, rg, nr, jobs, n, codes, bids, tot, ret, mp, aln);
    hsa_gpu_unlock();
    if (rc) hsa_gpu_fatal("GPU seed extension", rc);
    for (int j = 0; j < n; ++j) {
        memcpy(q[j]->aln, aln + 9 * (size_t)j, sizeof(bwt_aln1_t));
        *q[j]->max_pos_io = mp[j];
        q[j]->ret = ret[j];
        if (q[j]->owned) { free(q[j]->seq); free(q[j]->bid); }
        q[j]->seq = NULL; q[j]->bid = NULL;
    }
    free(rg); free(jobs); free(codes); free(bids); free(ret); free(mp); free(aln);
}

/* One sliced launch over the parked calls q[0..n) (slot[j]: the call's persistent slot):
 * each runs for at most SLICE_POPS pops.  Returns the number finished; a finished call
 * has its result applied and q[j]->started reset, an unfinished one stays parked. */
static int run_slices(hsa_index_t *ix, ext_req_t *const *q, const int32_t *slot, int n, int n_slots, uint8_t *done)
{
    hsa_regime_t *rg = (hsa_regime_t *)calloc((size_t)n, sizeof(hsa_regime_t));
    hsa_ext_job_t *jobs = (hsa_ext_job_t *)calloc((size_t)n, sizeof(hsa_ext_job_t));
    uint8_t *res = (uint8_t *)calloc((size_t)n, 1);
    size_t tot = 0;
    for (int j = 0; j < n; ++j) tot += (size_t)q[j]->n;
    uint8_t *codes = (uint8_t *)calloc(tot + 1, 1);
    int32_t *bids = (int32_t *)calloc(tot + 1, sizeof(int32_t));
    int nr = 0;
    size_t off = 0;
    for (int j = 0; j < n; ++j) {
        int r = 0;
        while (r < nr && memcmp(&rg[r], &q[j]->rg, sizeof(hsa_regime_t))) ++r;
        if (r == nr) rg[nr++] = q[j]->rg;
        hsa_ext_job_t *J = jobs + j;
        J->dir = q[j]->dir; J->len = q[j]->len; J->max_pos = q[j]->max_pos; J->regime = r;
        J->lo = q[j]->lo; J->n = q[j]->n; J->off = off;
        memcpy(J->aln, q[j]->aln, sizeof(bwt_aln1_t));     /* the caller's hit, unchanged until done */
        memcpy(codes + off, q[j]->seq, (size_t)q[j]->n);
        memcpy(bids + off, q[j]->bid, sizeof(int32_t) * (size_t)q[j]->n);
        off += (size_t)q[j]->n;
        res[j] = (uint8_t)q[j]->started;
    }
    int32_t *ret = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t *mp = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    uint32_t *aln = (uint32_t *)malloc(sizeof(bwt_aln1_t) * (size_t)n);
    hsa_gpu_lock();
    int rc = hsa_extend_sliced(ix, rg, nr, jobs, slot, res, n, codes, bids, tot, n_slots, SLICE_POPS, ret, mp, aln);
    hsa_gpu_unlock();
    if (rc) hsa_gpu_fatal("GPU seed extension", rc);
    int nd = 0;
    for (int j = 0; j < n; ++j) {
        done[j] = 0;
        if (ret[j] == HSA_EXT_CONT) { q[j]->started = 1; continue; }
        if (ret[j] == HSA_EXT_E_CAP) {                 /* more stack than a slot holds: alone */
            q[j]->started = 0;
            ext_req_t *one = q[j];
            run_reqs(ix, &one, 1);
        } else if (ret[j] < -1) {
            hsa_gpu_fatal("GPU seed extension (undefined in the reference)", ret[j]);
        } else {
            memcpy(q[j]->aln, aln + 9 * (size_t)j, sizeof(bwt_aln1_t));
            *q[j]->max_pos_io = mp[j];
            q[j]->ret = ret[j];
            if (q[j]->owned) { free(q[j]->seq); free(q[j]->bid); }
            q[j]->seq = NULL; q[j]->bid = NULL;
        }
        q[j]->started = 0;
        done[j] = 1;
        ++nd;
    }
    free(rg); free(jobs); free(res); free(codes); free(bids); free(ret); free(mp); free(aln);
    return nd;
}

static int extend(bwt_aux_t *aux, bwt_aln1_t *aln, int *max_pos, int dir)
{
    co_t *me = tl_co;
    if (me) {                             /* inside the runner: park the call and yield */
        fill_req(&me->req, aux, aln, max_pos, dir, me->len);
        me->req.started = 0;
        me->req.kind = 0;
        me->state = 1;
        if (!_setjmp(me->jb)) _longjmp(*tl_sched, 1);
        return me->req.ret;
    }
    ext_req_t q;                          /* a direct call: a batch of one */
    memset(&q, 0, sizeof q);
    fill_req(&q, aux, aln, max_pos, dir, -1);
    ext_req_t *qp = &q;
    run_reqs(hsa_gpu_index_of(aux->bi_bwt), &qp, 1);
    return q.ret;
}

/* bwt_extend_backward (bwtgap.c:640-649): extend aln backward, at least to *_left. */
int bwt_extend_backward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_left) { return extend(aux, aln, _left, 1); }

/* bwt_extend_foreward (bwtgap.c:654-663): extend aln forward, at least to *_right. */
int bwt_extend_foreward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_right) { return extend(aux, aln, _right, 0); }

extern __typeof__(bwt_extend_backward) hsa_own_extend_backward
    __attribute__((alias("bwt_extend_backward"), visibility("hidden")));

/* Whether the host's bwt_splice_match calls these extensions (the host linked
 * bwtext_gpu.o and weakened its own): only then does the batched runner pay. */
int hsa_splice_extend_active(void)
{
    int (*volatile resolved)(bwt_aux_t *, bwt_aln1_t *, int *) = bwt_extend_backward;
    return resolved == hsa_own_extend_backward;
}

#pragma weak hsa_splice_set_read
#pragma weak hsa_splice_table_width
#pragma weak hsa_splice_table_sa

/* bwt_cal_width on the GPU for n sequences of one type; w: 2 * (len + 1) words each */
static void widths_gpu(hsa_index_t *ix, int type, int n, const uint64_t *offs, const uint32_t *lens,
                       const uint8_t *codes, size_t codes_len, uint32_t *w)
{
    hsa_gpu_lock();
    const int rc = type == 1 ? hsa_width_batch(ix, (size_t)n, offs, lens, codes, codes_len, w)
                             : hsa_width0_batch(ix, (size_t)n, offs, lens, codes, codes_len, w);
    hsa_gpu_unlock();
    if (rc) hsa_gpu_fatal("GPU bwt_cal_width", rc);
}

/* bwt_cal_width (bwtaln.c:73-116): from the splice table of the thread's read, or one
 * GPU call. */
int bwt_cal_width(const Idx2BWT *bi_bwt, int len, const ubyte_t *str, bwt_width_t *width, int type)
{
    if (len < 0) len = 0;
    int ret = 0;
    if (hsa_splice_table_width && hsa_splice_table_width(bi_bwt, len, str, width, type == 1, &ret)) return ret;
    uint64_t off = 0;
    uint32_t l32 = (uint32_t)len;
    uint32_t *w = (uint32_t *)calloc(2 * ((size_t)len + 1), sizeof(uint32_t));
    widths_gpu(hsa_gpu_index_of(bi_bwt), type == 1, 1, &off, &l32, str, (size_t)len, w);
    for (int i = type == 1 ? 0 : 1; i <= len; ++i) { width[i].w = w[2 * i]; width[i].bid = (int)w[2 * i + 1]; }
    ret = (int)w[2 * len + 1];
    free(w);
    return ret;
}

extern __typeof__(bwt_cal_width) hsa_own_cal_width __attribute__((alias("bwt_cal_width"), visibility("hidden")));

int hsa_splice_width_active(void)
{
    int (*volatile resolved)(const Idx2BWT *, int, const ubyte_t *, bwt_width_t *, int) = bwt_cal_width;
    return resolved == hsa_own_cal_width;
}

/* ------------------------------------------------------------ SA -> position
 * The splice path's BWTRetrievePositionFromSAIndex calls (bwt_aln_corelate_check,
 * bwtgap.c:699, :712; check_site_by_intron_end, :615), redirected to
 * hsa_splice_sa_position by the host's link recipe (its bwtgap.o's reference renamed,
 * INTEGRATION.md; the SAM stage keeps the host's own).  Answers come from the read's
 * splice table (the ranges the correlation reads of every prefetched seed and anchor hit,
 * bwtgap_gpu.c), then from this table of the runner's earlier rounds; a lookup both miss
 * parks its coroutine, and each round's parked lookups are one GPU launch. */
typedef struct { uint32_t key, sid, ori, occ; } sa_ent_t;   /* key = sa index + 1 (0: empty) */
static sa_ent_t *g_sa;
static size_t g_sa_cap2, g_sa_n2;
static uint64_t g_sa_hits, g_sa_misses;
static pthread_rwlock_t g_sa_mu = PTHREAD_RWLOCK_INITIALIZER;

static size_t sa_slot(uint32_t key, size_t cap)
{
    return (size_t)((key * 0x9E3779B97F4A7C15ull) >> 20) & (cap - 1);
}

static void sa_put(uint32_t idx, const uint32_t o4[4])      /* caller holds g_sa_mu */
{
    if (2 * (g_sa_n2 + 1) > g_sa_cap2) {
        size_t cap = g_sa_cap2 ? 2 * g_sa_cap2 : 1u << 16;
        sa_ent_t *t = (sa_ent_t *)calloc(cap, sizeof(sa_ent_t));
        for (size_t i = 0; i < g_sa_cap2; ++i) {
            if (!g_sa[i].key) continue;
            size_t j = sa_slot(g_sa[i].key, cap);
            while (t[j].key) j = (j + 1) & (cap - 1);
            t[j] = g_sa[i];
        }
        free(g_sa);
        g_sa = t;
        g_sa_cap2 = cap;
    }
    const uint32_t key = idx + 1u;
    size_t j = sa_slot(key, g_sa_cap2);
    while (g_sa[j].key && g_sa[j].key != key) j = (j + 1) & (g_sa_cap2 - 1);
    if (g_sa[j].key) return;
    g_sa[j].key = key; g_sa[j].occ = o4[0]; g_sa[j].sid = o4[1]; g_sa[j].ori = o4[2];
    ++g_sa_n2;
}

static const sa_ent_t *sa_get(uint32_t idx)                 /* caller holds g_sa_mu */
{
    if (!g_sa_n2) return NULL;
    const uint32_t key = idx + 1u;
    for (size_t j = sa_slot(key, g_sa_cap2); g_sa[j].key; j = (j + 1) & (g_sa_cap2 - 1))
        if (g_sa[j].key == key) return g_sa + j;
    return NULL;
}

/* BWTRetrievePositionFromSAIndex's outputs (2BWT-Interface.c:329-361): the packed
 * position always, sequence id and 1-based position only when a block holds it. */
static void sa_write(uint32_t occ, uint32_t sid, uint32_t ori, unsigned int *sid_p, unsigned int *ori_p,
                     unsigned int *occ_p)
{
    *occ_p = occ;
    if (sid != 0xFFFFFFFFu) { *sid_p = sid; *ori_p = ori; }
}

void hsa_splice_sa_clear(void)
{
    pthread_rwlock_wrlock(&g_sa_mu);
    free(g_sa);
    g_sa = NULL;
    g_sa_cap2 = g_sa_n2 = 0;
    pthread_rwlock_unlock(&g_sa_mu);
}

void hsa_splice_sa_stats(uint64_t *hits, uint64_t *misses)
{
    pthread_rwlock_wrlock(&g_sa_mu);
    *hits = g_sa_hits; *misses = g_sa_misses;
    g_sa_hits = g_sa_misses = 0;
    pthread_rwlock_unlock(&g_sa_mu);
}

/* BWTRetrievePositionFromSAIndex (2BWT-Interface.c:329) for the splice path. */
void hsa_splice_sa_position(Idx2BWT *bi, unsigned int sa_index, unsigned int *seq_id, unsigned int *ori_pos,
                            unsigned int *occ_pos)
{
    uint32_t o3[3];
    if (hsa_splice_table_sa && hsa_splice_table_sa(bi, sa_index, o3)) {
        sa_write(o3[0], o3[1], o3[2], seq_id, ori_pos, occ_pos);
        return;
    }
    pthread_rwlock_rdlock(&g_sa_mu);
    const sa_ent_t *e = sa_get(sa_index);
    sa_ent_t v = e ? *e : (sa_ent_t){0, 0, 0, 0};
    if (e) __atomic_fetch_add(&g_sa_hits, 1, __ATOMIC_RELAXED);
    else __atomic_fetch_add(&g_sa_misses, 1, __ATOMIC_RELAXED);
    pthread_rwlock_unlock(&g_sa_mu);
    if (e) { sa_write(v.occ, v.sid, v.ori, seq_id, ori_pos, occ_pos); return; }
    co_t *me = tl_co;
    if (me) {                             /* park; the round's lookups are one launch */
        me->req.kind = 1;
        me->req.sa = sa_index;
        me->req.sid_p = seq_id; me->req.ori_p = ori_pos; me->req.occ_p = occ_pos;
        me->state = 1;
        if (!_setjmp(me->jb)) _longjmp(*tl_sched, 1);
        return;
    }
    const uint32_t one = sa_index;
    uint32_t o4[4];
    hsa_index_t *ix = hsa_gpu_index_of(bi);
    hsa_gpu_lock();
    const int rc = hsa_sa_position_batch(ix, 1, &one, o4);
    hsa_gpu_unlock();
    if (rc) hsa_gpu_fatal("GPU SA -> position", rc);
    sa_write(o4[0], o4[1], o4[2], seq_id, ori_pos, occ_pos);
}

/* gap_init_stack's layout (bwtgap.c:13-27): the host's splice code resets and reads it */
static gap_stack_t *stack_new(int n_stacks)
{
    gap_stack_t *s = (gap_stack_t *)calloc(1, sizeof(gap_stack_t));
    s->n_stacks = n_stacks;
    s->stacks = (gap_stack1_t *)calloc((size_t)n_stacks, sizeof(gap_stack1_t));
    for (int i = 0; i < n_stacks; ++i) {
        s->stacks[i].m_entries = 4;
        s->stacks[i].stack = (gap_entry_t *)calloc(4, sizeof(gap_entry_t));
    }
    return s;
}

static void stack_free(gap_stack_t *s)
{
    for (int i = 0; i < s->n_stacks; ++i) free(s->stacks[i].stack);
    free(s->stacks);
    free(s);
}

static void co_entry(void)
{
    co_t *me = tl_co;
    me->result = bwt_splice_match(&me->aux, &me->n_aln);
    me->state = 2;
    _longjmp(*tl_sched, 1);          /* never returns: the runner takes the next read */
}

/* Start coroutine c on read r: the aux bwa_cal_sa_reg_gap hands bwt_splice_match
 * (bwtaln.c:326-364: seq, len, rc_seq, strand 0, opt = local_opt of that read). */
static void co_start(co_t *c, int r, const hsa_splice_read_t *rd)
{
    c->read = r;
    c->state = 0;
    c->opt = rd->opt;
    c->len = rd->len;
    c->aux.opt = &c->opt;
    c->aux.seq = (ubyte_t *)rd->seq;
    c->aux.len = rd->len;
    c->aux.strand = 0;
    memset(c->aux.rc_seq, 0, (size_t)c->aux.max_len);
    for (int j = 0; j < rd->len; ++j) {
        const ubyte_t x = rd->seq[rd->len - 1 - j];
        c->aux.rc_seq[j] = x < 4 ? (ubyte_t)(3 - x) : x;
    }
    c->result = NULL;
    c->n_aln = 0;
    getcontext(&c->uc);
    c->uc.uc_stack.ss_sp = c->stack;
    c->uc.uc_stack.ss_size = CO_STACK;
    c->uc.uc_link = NULL;
    makecontext(&c->uc, co_entry, 0);
    c->entered = 0;
}

/* The coroutines (stacks, per-read buffers, the stack object the host's code sees) are
 * kept between calls: a batch's splice path is short, and mapping, guarding and
 * unmapping thousands of stacks per call cost as much as running them (and the
 * unmaps' TLB shootdowns grow with the runner's threads). */
static co_t *g_co;
static int g_co_n, g_co_len, g_co_stacks;
static pthread_mutex_t g_co_mu = PTHREAD_MUTEX_INITIALIZER;

static co_t *co_pool(int W, int max_len, int n_stacks)
{
    if (W > g_co_n) {
        co_t *p = (co_t *)realloc(g_co, sizeof(co_t) * (size_t)W);
        if (!p) { fprintf(stderr, "[hsa_splice_run] out of memory\n"); exit(1); }
        memset(p + g_co_n, 0, sizeof(co_t) * (size_t)(W - g_co_n));
        g_co = p;
        for (int k = g_co_n; k < W; ++k) {
            co_t *c = g_co + k;
            /* one guard page below each stack: an overflow faults instead of silently
             * corrupting the neighbouring coroutine's stack */
            void *m = mmap(NULL, CO_STACK + CO_GUARD, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                           -1, 0);
            if (m == MAP_FAILED || mprotect(m, CO_GUARD, PROT_NONE)) {
                fprintf(stderr, "[hsa_splice_run] cannot map a coroutine stack\n");
                exit(1);
            }
            c->stack = (char *)m + CO_GUARD;
        }
        g_co_n = W;
    }
    if (max_len > g_co_len || n_stacks != g_co_stacks) {
        const int len = max_len > g_co_len ? max_len : g_co_len;
        for (int k = 0; k < g_co_n; ++k) {
            co_t *c = g_co + k;
            if (c->aux.stack) stack_free(c->aux.stack);
            free(c->aux.width_back); free(c->aux.width_fore); free(c->aux.width_seed); free(c->aux.rc_seq);
            free(c->req.buf);
            c->aux.stack = NULL;
        }
        g_co_len = len;
        g_co_stacks = n_stacks;
    }
    for (int k = 0; k < W; ++k) {
        co_t *c = g_co + k;
        if (!c->aux.stack) {
            c->aux.width_back = (bwt_width_t *)calloc((size_t)g_co_len + 1, sizeof(bwt_width_t));
            c->aux.width_fore = (bwt_width_t *)calloc((size_t)g_co_len + 1, sizeof(bwt_width_t));
            c->aux.width_seed = (bwt_width_t *)calloc((size_t)g_co_len + 1, sizeof(bwt_width_t));
            c->aux.rc_seq = (ubyte_t *)calloc((size_t)g_co_len + 1, 1);
            c->aux.stack = stack_new(n_stacks);
            c->req.buf_cap = 5 * ((size_t)g_co_len + 4);    /* the largest window: the read and both bounds */
            c->req.buf = (uint8_t *)malloc(c->req.buf_cap);
        }
        c->read = -1;
        c->state = 0;
        c->entered = 0;
    }
    return g_co;
}

/* The coroutine pool made ahead of the first batch (hsa_gpu_attach): n coroutines, their
 * stacks mapped and the top pages of each touched, so that the first batch's splice
 * path does not pay the mappings and first-touch faults. */
void hsa_splice_warm(int n)
{
    if (n > CO_MAX) n = CO_MAX;
    pthread_mutex_lock(&g_co_mu);
    co_t *co = co_pool(n, 128, 1);
    for (int k = 0; k < n; ++k)
        memset((char *)co[k].stack + CO_STACK - (32u << 10), 0, 32u << 10);
    pthread_mutex_unlock(&g_co_mu);
}

/* One host thread of the runner: its coroutines, the reads they take from the shared
 * queue, and its own scheduling point (tl_sched). */
typedef struct runner_s runner_t;
typedef struct {
    runner_t *R;
    int id;
    co_t *co;                 /* this worker's coroutines: global slots [c0, c0 + W) */
    int W, c0, live;
    jmp_buf sched;
    pthread_t th;
} worker_t;

struct runner_s {
    const Idx2BWT *bi;
    hsa_index_t *ix;
    const hsa_splice_read_t *reads;
    bwt_aln1_t **out;
    int *n_out;
    int n, T;
    int next;                 /* the next read of the queue (atomic) */
    pthread_barrier_t bar;
    int done;                 /* set by the leader: no read is left anywhere */
    worker_t *w;
    /* the leader's round: parked calls of every worker */
    ext_req_t **pend;
    int32_t *pslot;
    uint8_t *pdone;
    co_t **pco;
    int *wide;
    uint32_t *sa_idx, *sa_o4;
    co_t **sa_co;
    long launches, calls, sa_launches;
    double t_gpu, t_setup, t_work;   /* t_work: the rounds' slowest worker, summed */
    double *busy;                    /* per worker, the round's coroutine time */
};

/* Run every runnable coroutine of worker w until it parks or finishes; a finished one
 * takes the next read of the queue at once. */
static void worker_round(worker_t *w)
{
    runner_t *R = w->R;
    tl_sched = &w->sched;
    for (volatile int k = 0; k < w->W; ++k) {       /* volatile: live across _setjmp */
        co_t *c = w->co + k;
        while (c->read >= 0 && c->state == 0) {
            tl_co = c;
            if (hsa_splice_set_read) hsa_splice_set_read(c->read);   /* its splice table entries */
            if (!_setjmp(w->sched)) {
                if (!c->entered) { c->entered = 1; setcontext(&c->uc); }
                _longjmp(c->jb, 1);
            }
            tl_co = NULL;
            if (hsa_splice_set_read) hsa_splice_set_read(-1);
            if (c->state == 2) {
                R->out[c->read] = c->result;
                R->n_out[c->read] = c->n_aln;
                const int r = __atomic_fetch_add(&R->next, 1, __ATOMIC_RELAXED);
                if (r < R->n) co_start(c, r, R->reads + r);
                else { c->read = -1; --w->live; }
            }
        }
    }
}

/* The leader's part of a round: one SA -> position launch and one sliced extension
 * launch (wide regimes: one hsa_extend_batch) over the parked calls of all workers. */
static void leader_round(runner_t *R)
{
    int np = 0, nsa = 0, nwide = 0, live = 0;
    for (int t = 0; t < R->T; ++t) {
        worker_t *w = R->w + t;
        live += w->live;
        for (int k = 0; k < w->W; ++k) {
            co_t *c = w->co + k;
            if (c->read < 0 || c->state != 1) continue;
            if (c->req.kind == 1) { R->sa_idx[nsa] = c->req.sa; R->sa_co[nsa++] = c; }
            else if (c->req.rg.n_stacks > HSA_EXT_SLICE_STACKS) { R->pco[nwide] = c; R->pend[nwide] = &c->req; ++nwide; }
        }
    }
    if (live == 0) { R->done = 1; return; }
    if (nsa > 0) {                    /* the round's SA -> position lookups: one launch */
        const double ts = hsa_now();
        hsa_gpu_lock();
        const int rc = hsa_sa_position_batch(R->ix, (size_t)nsa, R->sa_idx, R->sa_o4);
        hsa_gpu_unlock();
        if (rc) hsa_gpu_fatal("GPU SA -> position", rc);
        pthread_rwlock_wrlock(&g_sa_mu);
        for (int j = 0; j < nsa; ++j) {
            ext_req_t *q = &R->sa_co[j]->req;
            sa_write(R->sa_o4[4 * j], R->sa_o4[4 * j + 1], R->sa_o4[4 * j + 2], q->sid_p, q->ori_p, q->occ_p);
            sa_put(R->sa_idx[j], R->sa_o4 + 4 * j);
            R->sa_co[j]->state = 0;
        }
        pthread_rwlock_unlock(&g_sa_mu);
        R->t_gpu += hsa_now() - ts;
        ++R->sa_launches;
    }
    /* a call whose regime has more score LIFOs than a slice slot holds (n_stacks > 256,
     * e.g. -O 120) runs to completion in one hsa_extend_batch launch */
    if (nwide > 0) {
        const double tw = hsa_now();
        run_reqs(R->ix, R->pend, nwide);
        for (int j = 0; j < nwide; ++j) R->pco[j]->state = 0;
        R->t_gpu += hsa_now() - tw;
        R->calls += nwide;
        ++R->launches;
    }
    /* one sliced launch over every other parked extension (slot = its coroutine): the
     * finished ones resume, the others stay parked with their state on the device */
    int W = 0;
    for (int t = 0; t < R->T; ++t) {
        worker_t *w = R->w + t;
        for (int k = 0; k < w->W; ++k) {
            co_t *c = w->co + k;
            if (c->read >= 0 && c->state == 1 && c->req.kind == 0 && c->req.rg.n_stacks <= HSA_EXT_SLICE_STACKS) {
                R->pend[np] = &c->req; R->pslot[np] = w->c0 + k; R->pco[np] = c; ++np;
            }
        }
        W += w->W;
    }
    if (np == 0) return;
    const double tg = hsa_now();
    const int nd = run_slices(R->ix, R->pend, R->pslot, np, W, R->pdone);
    R->t_gpu += hsa_now() - tg;
    if (getenv("HSA_EXT_TRACE"))
        fprintf(stderr, "[hsa_splice_run] round %ld: %d parked, %d finished, %.3f ms\n", R->launches, np, nd,
                1e3 * (hsa_now() - tg));
    R->calls += nd;
    ++R->launches;
    for (int j = 0; j < np; ++j)
        if (R->pdone[j]) R->pco[j]->state = 0;
}

static void *worker_main(void *arg)
{
    worker_t *w = (worker_t *)arg;
    runner_t *R = w->R;
    for (;;) {
        const double t0 = hsa_now();
        worker_round(w);
        R->busy[w->id] = hsa_now() - t0;
        pthread_barrier_wait(&R->bar);
        if (w->id == 0) {
            double mx = 0.0;
            for (int t = 0; t < R->T; ++t) mx = R->busy[t] > mx ? R->busy[t] : mx;
            R->t_work += mx;
            leader_round(R);
        }
        pthread_barrier_wait(&R->bar);
        if (R->done) break;
    }
    tl_sched = NULL;
    return NULL;
}

static int runner_threads(int n)
{
    const char *e = getenv("HSA_SPLICE_THREADS");
    int t = e ? atoi(e) : 0;
    if (t > 0) return t < n ? t : n;        /* as asked (tests: several threads on few reads) */
    cpu_set_t cs;
    CPU_ZERO(&cs);
    t = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 1;
    if (t > 16) t = 16;                     /* one GPU's share of a shared host */
    const int by_reads = (n + 63) / 64;     /* at least 64 reads a thread */
    if (t > by_reads) t = by_reads;
    return t < 1 ? 1 : t;
}

/* bwt_splice_match for reads[0..n) (see the file comment): out[r] / n_out[r] are what
 * bwt_splice_match(aux of read r) returns.  T host threads run the reads as coroutines
 * (each thread its own; reads pulled from one queue), and every round's parked calls
 * of all threads go to the device in one launch.  Returns the number of GPU extension
 * launches. */
long hsa_splice_run(const Idx2BWT *bi, struct bwt_array_t *arr, int max_len, int n_stacks, int n,
                    const hsa_splice_read_t *reads, bwt_aln1_t **out, int *n_out)
{
    if (n <= 0) return 0;
    if (!bwt_splice_match) { for (int r = 0; r < n; ++r) { out[r] = NULL; n_out[r] = 0; } return 0; }
    runner_t R;
    memset(&R, 0, sizeof R);
    R.bi = bi; R.ix = hsa_gpu_index_of(bi); R.reads = reads; R.out = out; R.n_out = n_out; R.n = n;
    const int Wtot = n < CO_MAX ? n : CO_MAX;
    R.T = runner_threads(n);
    if (R.T > Wtot) R.T = Wtot;
    R.w = (worker_t *)calloc((size_t)R.T, sizeof(worker_t));
    const double t_setup = hsa_now();
    pthread_mutex_lock(&g_co_mu);
    co_t *co = co_pool(Wtot, max_len, n_stacks);
    for (int k = 0; k < Wtot; ++k) {
        co[k].aux.bi_bwt = (Idx2BWT *)bi;
        co[k].aux.arr = arr;
        co[k].aux.max_len = max_len;
    }
    /* coroutines split evenly over the threads; the first reads handed out in order */
    for (int t = 0, c0 = 0; t < R.T; ++t) {
        worker_t *w = R.w + t;
        const int W = Wtot / R.T + (t < Wtot % R.T);
        w->R = &R; w->id = t; w->co = co + c0; w->W = W; w->c0 = c0;
        c0 += W;
    }
    for (int k = 0; k < Wtot; ++k) {
        for (int t = 0; t < R.T; ++t)
            if (k >= R.w[t].c0 && k < R.w[t].c0 + R.w[t].W) { ++R.w[t].live; break; }
        co_start(co + k, k, reads + k);
    }
    R.next = Wtot;
    R.pend = (ext_req_t **)malloc(sizeof(ext_req_t *) * (size_t)Wtot);
    R.pslot = (int32_t *)malloc(sizeof(int32_t) * (size_t)Wtot);
    R.pdone = (uint8_t *)malloc((size_t)Wtot);
    R.pco = (co_t **)malloc(sizeof(co_t *) * (size_t)Wtot);
    R.sa_idx = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)Wtot);
    R.sa_o4 = (uint32_t *)malloc(sizeof(uint32_t) * 4 * (size_t)Wtot);
    R.sa_co = (co_t **)malloc(sizeof(co_t *) * (size_t)Wtot);
    R.busy = (double *)calloc((size_t)R.T, sizeof(double));
    const double t_run = hsa_now();
    R.t_setup = t_run - t_setup;
    pthread_barrier_init(&R.bar, NULL, (unsigned)R.T);
    for (int t = 1; t < R.T; ++t)
        if (pthread_create(&R.w[t].th, NULL, worker_main, R.w + t)) {
            fprintf(stderr, "[hsa_splice_run] cannot start a runner thread\n");
            exit(1);
        }
    worker_main(R.w);
    for (int t = 1; t < R.T; ++t) pthread_join(R.w[t].th, NULL);
    pthread_barrier_destroy(&R.bar);
    pthread_mutex_unlock(&g_co_mu);
    free(R.w); free(R.pend); free(R.pslot); free(R.pdone); free(R.pco); free(R.sa_idx); free(R.sa_o4);
    free(R.sa_co); free(R.busy);
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] splice runner: %d reads on %d host threads, %ld extension calls in %ld launches, %ld SA "
                        "lookup launches: %.3f s in the launches (copies included), %.3f s of host splice code "
                        "(rounds' slowest worker %.3f s, set-up %.3f s)\n", n, R.T, R.calls, R.launches, R.sa_launches,
                R.t_gpu, hsa_now() - t_run - R.t_gpu, R.t_work, R.t_setup);
    return R.launches;
}
