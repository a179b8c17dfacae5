/*
 * bwtsam_gpu.c -- drop-in generate_sam_se_core (bwtse.c:884-932): the SAM stage of one
 * read batch on several host threads, printing the reference's bytes in the reference's
 * order.
 *
 * The reference runs the stage single-threaded after every batch (bwtaln.c:514):
 *   1. bwt_aln2seq_core per read (bwtse.c:21-113): picks one of the equal-best hits with
 *      drand48 (bwtse.c:44, :51) and samples the extra positions (bwtse.c:97);
 *   2. bwa_cal_pac_pos (bwtse.c:350): SA -> position (ours runs it on the GPU,
 *      bwtse_gpu.c);
 *   3. bwa_refine_gapped (bwtse.c:536): CIGAR by banded global DP for gapped hits, MD;
 *   4. bwa_print_sam1 (bwtse.c:677) of every read with a hit.
 * Steps 3 and 4 are per-read functions of the read alone; step 1 is too, except for the
 * process-wide drand48 sequence it consumes in read order.
 *
 * drand48 by jump-ahead.  A sequential pre-pass walks the reads in order with the
 * draw logic of step 1 only (which draws a read makes depends on the values drawn, so
 * the walk evaluates them; it writes nothing) and records the 48-bit generator state
 * at the start of every read.  Step 1 then runs on N threads, read r drawing with
 * erand48() from its recorded state: erand48 and drand48 are the same generator and
 * the same conversion to double (glibc: both are __erand48_r with the process's
 * multiplier and addend, which the reference never changes), so every read sees the
 * numbers the reference would have drawn for it.  At the end the process's drand48
 * state is set (seed48) to where the reference leaves it: the next batch, and any
 * other drand48 caller, continue the same sequence.
 *
 * Output.  Each thread prints its reads into per-chunk buffers (chunks of CHUNK reads
 * taken dynamically: gapped reads cost a DP each); the chunks are written to stdout in
 * read order.  The printing restates bwa_print_sam1 for the single-end case (mate ==
 * NULL, bwtse.c:924) byte for byte.  Guard: on the first batch of the process the
 * host's own bwa_print_sam1 prints the first GUARD_READS reads into a memory stream
 * (stdout swapped while no other thread runs) and the restatement must print the
 * same bytes; otherwise the stage falls back to the host's printing, sequentially,
 * for the rest of the process (logged once).  Steps 2 and 3 are the host's own
 * functions (bwa_cal_pac_pos: ours or the host's, whichever the program links;
 * bwa_refine_gapped on disjoint chunks of reads).
 *
 * HSA_SAM_THREADS=n sets the thread count (default: the CPUs this process may run on,
 * at most 16); n = 1 runs the same code on the calling thread.  HSA_SAM_CHUNK=m sets
 * the reads per chunk (default 2048; tests use small chunks).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/hsa_bwtaln.h"

/* the host's functions and data this stage uses (bwtse.c, bwaseqio.c, bwtse.c:15) */
#pragma weak bwa_cal_pac_pos
#pragma weak bwa_refine_gapped
#pragma weak bwa_print_sam1
#pragma weak seq_reverse
#pragma weak bwt_rg_id
extern void bwa_refine_gapped(const HSP *hsp, int n_seqs, bwa_seq_t *seqs);
extern void bwa_print_sam1(const HSP *hsp, bwa_seq_t *p, const bwa_seq_t *mate, int mode, int max_top2);
extern void seq_reverse(int len, ubyte_t *seq, int is_comp);
extern char *bwt_rg_id;

/* monotonic seconds (this file links on its own into a CPU-only host: ref.mk HSA_sam) */
static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

#define BWA_TYPE_MATESW 3
#define SAM_FSR 16
#define CHUNK_DEFAULT 2048
#define GUARD_READS 256
#define MAX_THREADS 64

/* ------------------------------------------------------------------ step 1 */

/* the draws bwt_aln2seq_core makes for one read (bwtse.c:38-110), without its writes:
 * advances xs past them */
static void aln2seq_draws(const bwa_seq_t *s, int n_multi, unsigned short xs[3])
{
    const int n_aln = s->n_aln;
    const bwt_aln1_t *aln = s->aln;
    if (n_aln == 0) return;
    int i, cnt;
    const int best = aln[0].score;
    for (i = cnt = 0; i < n_aln; ++i) {                                   /* :40-55 */
        const bwt_aln1_t *p = aln + i;
        if (p->score > best) break;
        if (erand48(xs) * (p->l - p->k + 1 + cnt) > (double)cnt) (void)erand48(xs);
        cnt += p->l - p->k + 1;
    }
    if (n_multi) {                                                        /* :62-111 */
        int k, n_occ;
        for (k = n_occ = 0; k < n_aln; ++k) n_occ += aln[k].l - aln[k].k + 1;
        if (n_occ > n_multi + 1) return;
        int rest = n_occ > n_multi + 1 ? n_multi + 1 : n_occ;
        for (k = 0; k < n_aln; ++k) {
            const bwt_aln1_t *q = aln + k;
            if (q->l - q->k + 1 <= rest) { rest -= q->l - q->k + 1; continue; }
            for (int j = rest; j > 0; --j) (void)erand48(xs);             /* :96-106: one draw per sample */
            break;
        }
    }
}

/* bwt_aln2seq_core (bwtse.c:21-113), drawing from xs; same writes, same arithmetic types */
static void aln2seq(bwa_seq_t *s, int set_main, int n_multi, unsigned short xs[3])
{
    int i, cnt, best;
    const int n_aln = s->n_aln;
    bwt_aln1_t *aln = s->aln;
    if (n_aln == 0) {
        s->type = BWA_TYPE_NO_MATCH;
        s->c1 = s->c2 = 0;
        return;
    }
    if (s->aln->type == BWA_TYPE_SPLICING && s->n_aln == 1)              /* :32-34 */
        s->type = (s->aln->l - s->aln->k + 1 > 1) ? BWA_TYPE_REPEAT : BWA_TYPE_UNIQUE;
    if (set_main) {
        best = aln[0].score;
        for (i = cnt = 0; i < n_aln; ++i) {
            const bwt_aln1_t *p = aln + i;
            if (p->score > best) break;
            if (erand48(xs) * (p->l - p->k + 1 + cnt) > (double)cnt) {
                s->n_mm = p->n_mm; s->n_gapo = p->n_gapo; s->n_gape = p->n_gape;
                s->score = p->score; s->start = p->start; s->end = p->end;
                s->sa = p->k + (bwtint_t)((p->l - p->k + 1) * erand48(xs));
                s->strand = p->strand;
            }
            cnt += p->l - p->k + 1;
        }
        s->c1 = cnt;
        for (; i < n_aln; ++i) cnt += aln[i].l - aln[i].k + 1;
        s->c2 = cnt - s->c1;
        s->type = s->c1 > 1 ? BWA_TYPE_REPEAT : BWA_TYPE_UNIQUE;
    }
    if (n_multi) {
        int k, rest, n_occ, z = 0;
        for (k = n_occ = 0; k < n_aln; ++k) n_occ += aln[k].l - aln[k].k + 1;
        if (s->multi) free(s->multi);
        if (n_occ > n_multi + 1) { s->multi = 0; s->n_multi = 0; return; }
        rest = n_occ > n_multi + 1 ? n_multi + 1 : n_occ;
        s->multi = (bwt_multi1_t *)calloc(rest, sizeof(bwt_multi1_t));
        for (k = 0; k < n_aln; ++k) {
            const bwt_aln1_t *q = aln + k;
            if (q->l - q->k + 1 <= rest) {
                for (bwtint_t l = q->k; l <= q->l; ++l) {
                    s->multi[z].start = q->start; s->multi[z].end = q->end; s->multi[z].strand = q->strand;
                    s->multi[z].sa = l; s->multi[z].gap = q->n_gapo + q->n_gape; s->multi[z++].mm = q->n_mm;
                }
                rest -= q->l - q->k + 1;
            } else {                                                      /* random sample (:93-108) */
                int j, ii;
                for (j = rest, ii = q->l - q->k + 1; j > 0; --j) {
                    double p = 1.0, x = erand48(xs);
                    while (x < p) p -= p * j / (ii--);
                    s->multi[z].start = q->start; s->multi[z].end = q->end; s->multi[z].strand = q->strand;
                    s->multi[z].sa = q->l - ii; s->multi[z].gap = q->n_gapo + q->n_gape; s->multi[z++].mm = q->n_mm;
                }
                break;
            }
        }
        s->n_multi = z;
    }
}

/* ------------------------------------------------------------------ step 4 */

typedef struct { char *s; size_t n, cap; } sbuf_t;

static void sb_grow(sbuf_t *b, size_t add)
{
    if (b->n + add <= b->cap) return;
    size_t c = b->cap ? b->cap : 4096;
    while (c < b->n + add) c *= 2;
    char *p = (char *)realloc(b->s, c);
    if (!p) { fprintf(stderr, "[generate_sam_se_core] out of host memory\n"); exit(1); }
    b->s = p; b->cap = c;
}
static inline void sb_c(sbuf_t *b, char c) { sb_grow(b, 1); b->s[b->n++] = c; }
static inline void sb_s(sbuf_t *b, const char *s)
{
    const size_t l = strlen(s);
    sb_grow(b, l);
    memcpy(b->s + b->n, s, l);
    b->n += l;
}
/* printf's %d */
static inline void sb_d(sbuf_t *b, int v)
{
    char t[12];
    int k = 0;
    unsigned u = v < 0 ? 0u - (unsigned)v : (unsigned)v;
    do { t[k++] = (char)('0' + u % 10); u /= 10; } while (u);
    sb_grow(b, (size_t)k + 1);
    if (v < 0) b->s[b->n++] = '-';
    while (k) b->s[b->n++] = t[--k];
}

/* bwa_print_sam1 (bwtse.c:677-824) with mate == NULL, for a read with a hit (the
 * stage skips the others, bwtse.c:922-923).  The reference passes bit-fields of
 * uint64_t (c1, c2) to %d: the low 32 bits as int, which is what the casts give. */
static void print_sam1(sbuf_t *b, const HSP *hsp, bwa_seq_t *p, int mode, int max_top2)
{
    int flag = p->extra_flag, j;
    if (p->strand) flag |= SAM_FSR;
    sb_s(b, p->name); sb_c(b, '\t'); sb_d(b, flag); sb_c(b, '\t'); sb_s(b, hsp->chrName[(int)p->seq_id]); sb_c(b, '\t');
    sb_d(b, (int)p->ori_pos); sb_c(b, '\t'); sb_d(b, (int)p->mapQ); sb_c(b, '\t');
    if (p->cigar) {
        for (j = 0; j != p->n_cigar; ++j) {
            sb_d(b, (int)(p->cigar[j] & 0x0fffffffu));
            sb_c(b, "MIDNSHP=X"[p->cigar[j] >> 28]);
        }
    } else {
        sb_d(b, (int)p->len); sb_c(b, 'M');
    }
    sb_s(b, "\t*\t0\t0\t");
    const int fl = (int)p->full_len;
    sb_grow(b, (size_t)fl + 1);
    if (p->strand == 0)
        for (j = 0; j != fl; ++j) b->s[b->n++] = "ACGTN"[(int)p->seq[j]];
    else
        for (j = 0; j != fl; ++j) b->s[b->n++] = "TGCAN"[p->seq[fl - 1 - j]];
    b->s[b->n++] = '\t';
    if (p->qual) {
        if (p->strand) seq_reverse((int)p->len, p->qual, 0);
        sb_s(b, (const char *)p->qual);
    } else sb_c(b, '*');
    if (&bwt_rg_id && bwt_rg_id) { sb_s(b, "\tRG:Z:"); sb_s(b, bwt_rg_id); }
    if (p->bc[0]) { sb_s(b, "\tBC:Z:"); sb_s(b, p->bc); }
    if (p->clip_len < (int)p->full_len) { sb_s(b, "\tXC:i:"); sb_d(b, p->clip_len); }
    sb_s(b, "\tXT:A:"); sb_c(b, "NURMS"[p->type]);
    sb_s(b, (mode & BWA_MODE_COMPREAD) ? "\tNM:i:" : "\tCM:i:"); sb_d(b, (int)p->nm);
    if (p->type != BWA_TYPE_MATESW) {
        sb_s(b, "\tX0:i:"); sb_d(b, (int)(uint32_t)p->c1);
        if (p->c1 <= max_top2) { sb_s(b, "\tX1:i:"); sb_d(b, (int)(uint32_t)p->c2); }   /* bwtse.c:775, as written */
    }
    sb_s(b, "\tXM:i:"); sb_d(b, (int)p->n_mm);
    sb_s(b, "\tXO:i:"); sb_d(b, (int)p->n_gapo);
    sb_s(b, "\tXG:i:"); sb_d(b, (int)(p->n_gapo + p->n_gape));
    if (p->md) { sb_s(b, "\tMD:Z:"); sb_s(b, p->md); }
    if (p->n_multi) {
        sb_s(b, "\tXA:Z:");
        for (int i = 0; i < p->n_multi; ++i) {
            const bwt_multi1_t *q = p->multi + i;
            sb_s(b, hsp->chrName[q->seq_id]); sb_c(b, ','); sb_c(b, q->strand ? '-' : '+'); sb_d(b, (int)q->ori_pos);
            if (q->cigar) {
                for (int k = 0; k < (int)q->n_cigar; ++k) {
                    sb_d(b, (int)(q->cigar[k] & 0x0fffffffu));
                    sb_c(b, "MIDNS"[q->cigar[k] >> 28]);
                }
            } else {
                sb_c(b, ','); sb_d(b, (int)(q->gap + q->mm)); sb_c(b, ';');
            }
        }
    }
    sb_c(b, '\n');
}

/* ------------------------------------------------------------------ the stage */

typedef struct {
    int phase;                          /* 1: step 1; 2: steps 3 + 4 */
    bwa_seq_t *seqs;
    int n, n_occ;
    const unsigned short *xs;           /* 3 per read: drand48 state at the read's start */
    const HSP *hsp;
    int mode, max_top2;
    sbuf_t *out;                        /* one per chunk */
    int chunk;                          /* reads per chunk */
    int next;                           /* the next chunk (atomic) */
} sam_job_t;

static void *sam_worker(void *arg)
{
    sam_job_t *j = (sam_job_t *)arg;
    const int n_chunks = (j->n + j->chunk - 1) / j->chunk;
    for (;;) {
        const int c = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (c >= n_chunks) break;
        const int r0 = c * j->chunk, r1 = r0 + j->chunk < j->n ? r0 + j->chunk : j->n;
        if (j->phase == 1) {
            for (int r = r0; r < r1; ++r) {
                bwa_seq_t *p = j->seqs + r;
                if (p->n_aln == 2 && p->aln->type == BWA_TYPE_SPLICING) { p->type = BWA_TYPE_SPLICING; continue; }
                unsigned short xs[3] = {j->xs[3 * r], j->xs[3 * r + 1], j->xs[3 * r + 2]};
                aln2seq(p, 1, j->n_occ, xs);
            }
        } else {
            bwa_refine_gapped(j->hsp, r1 - r0, j->seqs + r0);
            sbuf_t *b = j->out + c;
            for (int r = r0; r < r1; ++r)
                if (j->seqs[r].type != BWA_TYPE_NO_MATCH) print_sam1(b, j->hsp, j->seqs + r, j->mode, j->max_top2);
        }
    }
    return NULL;
}

static void run_phase(sam_job_t *j, int nt)
{
    pthread_t th[MAX_THREADS];
    int started[MAX_THREADS] = {0};
    j->next = 0;
    for (int k = 1; k < nt; ++k) started[k] = pthread_create(&th[k], NULL, sam_worker, j) == 0;
    sam_worker(j);
    for (int k = 1; k < nt; ++k) if (started[k]) pthread_join(th[k], NULL);
}

static int sam_threads(void)
{
    const char *e = getenv("HSA_SAM_THREADS");
    int n = e ? atoi(e) : 0;
    if (n <= 0) {
        cpu_set_t cs;
        n = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 1;
        if (n > 16) n = 16;
    }
    return n < 1 ? 1 : n > MAX_THREADS ? MAX_THREADS : n;
}

/* The guard (first batch of the process): the host's bwa_print_sam1, on copies of the
 * first GUARD_READS reads with a hit, must print the bytes the restatement printed for
 * them (the prefix of chunk 0's buffer).  The restatement has already reversed the
 * quality strings of reverse-strand reads (bwtse.c:747-748); the copies get them back as
 * they were before printing.  Returns 0 when equal, 1 when not, 2 when the chunk has no
 * read with a hit (nothing compared: the next batch is checked). */
static int print_guard(const HSP *hsp, const bwa_seq_t *seqs, int n, int chunk, const sbuf_t *chunk0, int mode,
                       int max_top2)
{
    char *host = NULL;
    size_t hl = 0;
    FILE *ms = open_memstream(&host, &hl);
    if (!ms) return -1;
    fflush(stdout);
    FILE *save = stdout;
    stdout = ms;
    for (int i = 0, k = 0; i < n && i < chunk && k < GUARD_READS; ++i) {
        if (seqs[i].type == BWA_TYPE_NO_MATCH) continue;
        ++k;
        bwa_seq_t h = seqs[i];
        ubyte_t *q = NULL;
        if (h.qual) {
            const size_t ql = strlen((const char *)h.qual) + 1;
            q = (ubyte_t *)malloc(ql);
            memcpy(q, h.qual, ql);
            if (h.strand) seq_reverse((int)h.len, q, 0);
            h.qual = q;
        }
        bwa_print_sam1(hsp, &h, NULL, mode, max_top2);
        free(q);
    }
    stdout = save;
    fclose(ms);
    const int bad = hl == 0 ? 2 : hl > chunk0->n || memcmp(host, chunk0->s, hl) != 0;
    free(host);
    return bad;
}

void generate_sam_se_core(Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, gap_opt_t *opt, int n_occ)
{
    static int guard_state = 0;         /* 0: unchecked; 1: the restatement prints; -1: the host's function */
    if (!bwa_cal_pac_pos || !bwa_refine_gapped || !seq_reverse) {
        fprintf(stderr, "[generate_sam_se_core] the host lacks bwa_cal_pac_pos / bwa_refine_gapped / seq_reverse\n");
        exit(1);
    }
    const int nt = sam_threads();
    const double t0 = now_s();
    /* step 1's drand48 states: the process's state now, then each read's draws in order */
    unsigned short *xs = (unsigned short *)malloc(sizeof(unsigned short) * 3 * ((size_t)n_seqs + 1));
    unsigned short cur[3] = {0, 0, 0};
    {
        const unsigned short *old = seed48(cur);    /* reads the state; put back at once */
        memcpy(cur, old, sizeof cur);
        seed48(cur);
    }
    for (int i = 0; i < n_seqs; ++i) {
        memcpy(xs + 3 * i, cur, sizeof cur);
        const bwa_seq_t *p = seqs + i;
        if (p->n_aln == 2 && p->aln->type == BWA_TYPE_SPLICING) continue;   /* bwtse.c:901-905: no draws */
        aln2seq_draws(p, n_occ, cur);
    }
    const double tp = now_s();
    sam_job_t job;
    memset(&job, 0, sizeof job);
    job.seqs = seqs; job.n = n_seqs; job.n_occ = n_occ; job.xs = xs; job.hsp = bi_bwt->hsp;
    job.mode = opt->mode; job.max_top2 = opt->max_top2;
    const char *ce = getenv("HSA_SAM_CHUNK");
    job.chunk = ce && atoi(ce) > 0 ? atoi(ce) : CHUNK_DEFAULT;
    job.phase = 1;
    run_phase(&job, nt);
    seed48(cur);                                    /* where the reference's draws leave it */
    free(xs);
    const double t1 = now_s();
    fprintf(stderr, "[bwa_aln_core] convert to sequence coordinate... ");
    bwa_cal_pac_pos(bi_bwt, n_seqs, seqs, opt->max_diff, opt->fnr);
    const double t2 = now_s();
    fprintf(stderr, "%.2f sec\n", t2 - t0);

    fprintf(stderr, "[bwa_aln_core] refine gapped alignment... ");
    const int n_chunks = (n_seqs + job.chunk - 1) / job.chunk;
    job.out = (sbuf_t *)calloc((size_t)n_chunks + 1, sizeof(sbuf_t));
    job.phase = 2;
    if (guard_state >= 0) run_phase(&job, nt);
    else {
        bwa_refine_gapped(bi_bwt->hsp, n_seqs, seqs);
    }
    const double t3 = now_s();
    fprintf(stderr, "%.2f sec\n", t3 - t2);
    fprintf(stderr, "[bwa_aln_core] print alignment... ");
    if (guard_state == 0 && n_chunks > 0) {
        if (!bwa_print_sam1) guard_state = 1;       /* nothing to compare with */
        else {
            const int g = print_guard(bi_bwt->hsp, seqs, n_seqs, job.chunk, job.out, opt->mode, opt->max_top2);
            guard_state = g == 0 ? 1 : g == 2 ? 0 : -1;
            if (guard_state < 0) {
                fprintf(stderr, "\n[hsa] the host's bwa_print_sam1 prints other bytes than bwtse.c:677 does: SAM "
                                "lines come from the host's function, on one thread, from now on\n");
                for (int r = 0; r < n_seqs; ++r)    /* the quality strings as they were before printing */
                    if (seqs[r].type != BWA_TYPE_NO_MATCH && seqs[r].strand && seqs[r].qual)
                        seq_reverse((int)seqs[r].len, seqs[r].qual, 0);
            }
        }
    }
    if (guard_state >= 0) {
        for (int c = 0; c < n_chunks; ++c)
            if (job.out[c].n && fwrite(job.out[c].s, 1, job.out[c].n, stdout) != job.out[c].n) {
                fprintf(stderr, "[generate_sam_se_core] fwrite to stdout failed\n");
                exit(1);
            }
    } else {
        for (int r = 0; r < n_seqs; ++r)
            if (seqs[r].type != BWA_TYPE_NO_MATCH) bwa_print_sam1(bi_bwt->hsp, seqs + r, NULL, opt->mode, opt->max_top2);
    }
    for (int c = 0; c < n_chunks; ++c) free(job.out[c].s);
    free(job.out);
    const double t4 = now_s();
    fprintf(stderr, "%.2f sec\n", t4 - t3);
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] SAM stage of %d reads on %d threads: drand48 walk %.1f ms, hit choice %.1f ms, SA -> "
                        "position %.1f ms, refine + print %.1f ms, write %.1f ms, total %.1f ms\n", n_seqs, nt,
                1e3 * (tp - t0), 1e3 * (t1 - tp), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3), 1e3 * (t4 - t0));
}
