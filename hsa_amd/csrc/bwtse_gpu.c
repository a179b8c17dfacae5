/*
 * bwtse_gpu.c -- host side of the drop-in bwa_cal_pac_pos (bwtse.c:350-369): the SAM
 * stage's SA -> position step with the SA lookups batched on the GPU.
 *
 * The reference walks each read and calls BWTRetrievePositionFromSAIndex
 * (2BWT-Interface.c:329) once for its SA value (bwa_cal_pac_pos_core, bwtse.c:139-148),
 * once per extra hit position (bwtse.c:359-365) and, for a spliced read
 * (bwt_aln2pos_splicing, bwtse.c:295-348), once for each of the first 50 rows of both
 * segments' intervals: up to saInterval - 1 dependent rank queries each (BWTSaValue,
 * BWT.c:1195).  Here those lookups are gathered in the order the reference makes them,
 * answered by one hsa_sa_position_batch launch (k_sa_position, hsa_sa.hip), and written
 * back with the same per-read updates in the same order: mapQ before and after the
 * position (the host's bwa_approx_mapQ), seq_id and ori_pos only when a block holds the
 * position, the duplicate-position filter of the extra hits, and for spliced reads the
 * reference's pairing of the two segments' positions (bwt_combine_segment_splice,
 * bwtse.c:197-235, with its own quicksort qsort_for_bwt, bwtse.c:169-192, restated so
 * that equal positions end up in the same order).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hsa_bwtaln.h"
#include "bwtaln_gpu.h"

/* the host's own functions this step calls (bwtse.c:122, bwtaln.c:46) */
#pragma weak bwa_approx_mapQ
#pragma weak bwa_cal_maxdiff
extern int bwa_approx_mapQ(const bwa_seq_t *p, int mm);
extern int bwa_cal_maxdiff(int l, double err, double thres);

#define BWA_AVG_ERR 0.02
#define NOT_FOUND 0xffffffffu

_Static_assert(sizeof(bwt_multi1_t) == 40, "bwt_multi1_t layout");

/* BWTRetrievePositionFromSAIndex's outputs from one k_sa_position record (SA value,
 * seq id, 1-based position, packed position); seq_id / ori_pos stay as they are when
 * no block holds the position, as in the reference (2BWT-Interface.c:342-356) */
static void put_pos(const uint32_t *r, uint32_t *seq_id, uint32_t *ori_pos, uint32_t *occ_pos)
{
    *occ_pos = r[3];
    if (r[1] != NOT_FOUND) { *seq_id = r[1]; *ori_pos = r[2]; }
}

/* qsort_for_bwt (bwtse.c:169-192): the reference's quicksort by occ_pos, pivot the first
 * element; restated step for step, since the order of equal positions is its own */
static void sort_occ(bwt_multi1_t *m, int l, int u)
{
    if (l >= u) return;
    const bwtint_t pv = m[l].occ_pos;        /* m[l] stays in place until the final swap */
    int i = l, j = u + 1;
    for (;;) {
        do ++i; while (i <= u && m[i].occ_pos < pv);
        do --j; while (m[j].occ_pos > pv);
        if (i > j) break;
        bwt_multi1_t t = m[i]; m[i] = m[j]; m[j] = t;
    }
    bwt_multi1_t t = m[l]; m[l] = m[j]; m[j] = t;
    sort_occ(m, l, j - 1);
    sort_occ(m, j + 1, u);
}

/* bwt_combine_segment_splice (bwtse.c:197-235): the pairs (first segment, second
 * segment) at the shortest distance in (50, 50 000), moved to the front two by two */
static int combine_segments(bwt_multi1_t *multi, int n_multi)
{
    int n_res = 0;
    bwtint_t shortest = 0xffffffffu;
    if (n_multi == 2) return 1;
    sort_occ(multi, 0, n_multi - 1);
    for (int i = 0; i < n_multi - 1; ++i) {
        bwt_multi1_t *t = multi + i;
        if (t->aln_id != 0) continue;
        if (t->aln_id == (t + 1)->aln_id || t->seq_id != (t + 1)->seq_id || (t + 1)->occ_pos - t->occ_pos > shortest)
            continue;
        const bwtint_t d = (t + 1)->occ_pos - t->occ_pos;
        if (d < 50 || d > 50000) continue;
        if (d < shortest) {
            shortest = d;
            n_res = 1;
            if (i == 0) continue;
        } else if (d == shortest) n_res += 1;
        memmove(multi + (n_res - 1) * 2, t, sizeof(bwt_multi1_t) * 2);
    }
    return n_res;
}

/* the SA rows bwt_aln2pos_splicing looks up for segment a (bwtse.c:320): k, k + 1, ...
 * while <= l and < k + 50, in u32 arithmetic */
static size_t splice_rows(const bwt_aln1_t *a)
{
    size_t n = 0;
    for (bwtint_t s = a->k; s <= a->l && s < a->k + 50; ++s) ++n;
    return n;
}

void bwa_cal_pac_pos(const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seq, int max_mm, float fnr)
{
    if (!bwa_approx_mapQ || !bwa_cal_maxdiff) {
        fprintf(stderr, "[bwa_cal_pac_pos] the host lacks bwa_approx_mapQ / bwa_cal_maxdiff\n");
        exit(1);
    }
    /* the lookups of bwtse.c:352-366 in the order the reference makes them */
    size_t n = 0;
    for (int i = 0; i < n_seqs; ++i) {
        const bwa_seq_t *p = seq + i;
        if (p->type == BWA_TYPE_SPLICING) {
            if (p->n_aln == 2) n += splice_rows(p->aln) + splice_rows(p->aln + 1);
            continue;
        }
        if (p->type == BWA_TYPE_UNIQUE || p->type == BWA_TYPE_REPEAT) ++n;
        if (p->n_multi > 0) n += (size_t)p->n_multi;
    }
    uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    uint32_t *res = (uint32_t *)malloc(sizeof(uint32_t) * 4 * (n + 1));
    size_t q = 0;
    for (int i = 0; i < n_seqs; ++i) {
        const bwa_seq_t *p = seq + i;
        if (p->type == BWA_TYPE_SPLICING) {
            if (p->n_aln == 2)
                for (int a = 0; a < 2; ++a)
                    for (bwtint_t s = p->aln[a].k; s <= p->aln[a].l && s < p->aln[a].k + 50; ++s) idx[q++] = s;
            continue;
        }
        if (p->type == BWA_TYPE_UNIQUE || p->type == BWA_TYPE_REPEAT) idx[q++] = p->sa;
        for (int j = 0; j < p->n_multi; ++j) idx[q++] = p->multi[j].sa;
    }
    if (n > 0) {
        hsa_index_t *ix = hsa_gpu_index_of(bi_bwt);
        hsa_gpu_lock();
        const int rc = hsa_sa_position_batch(ix, n, idx, res);
        hsa_gpu_unlock();
        if (rc) hsa_gpu_fatal("GPU SA -> position", rc);
    }
    q = 0;
    for (int i = 0; i < n_seqs; ++i) {
        bwa_seq_t *p = seq + i;
        if (p->type == BWA_TYPE_SPLICING) {                      /* bwt_aln2pos_splicing, bwtse.c:295-348 */
            if (p->n_aln != 2) continue;
            p->strand = p->aln->strand;
            bwtint_t nm = p->aln->l - p->aln->k + (p->aln + 1)->l - (p->aln + 1)->k + 2;
            nm = nm >= 100 ? 100 : nm;
            const size_t rows = splice_rows(p->aln) + splice_rows(p->aln + 1);
            /* calloc(nm) in the reference; never fewer entries than it writes here */
            bwt_multi1_t *multi = (bwt_multi1_t *)calloc(nm > rows ? nm : rows, sizeof(bwt_multi1_t));
            p->c2 = p->c1 = nm;
            int cnt = 0;
            for (int a = 0; a < 2; ++a) {
                const bwt_aln1_t *al = p->aln + a;
                const int mm = al->n_mm + al->n_gapo + al->n_gape;
                for (bwtint_t s = al->k; s <= al->l && s < al->k + 50; ++s, ++cnt) {
                    bwt_multi1_t *m = multi + cnt;
                    put_pos(res + 4 * q++, &m->seq_id, &m->ori_pos, &m->occ_pos);
                    m->strand = al->strand; m->start = al->start; m->end = al->end;
                    m->aln_id = (unsigned)a; m->mm = mm;
                }
            }
            const int n_splice = combine_segments(multi, cnt);
            p->n_multi = n_splice;
            if (n_splice == 0) {
                p->type = BWA_TYPE_NO_MATCH;
                free(multi);
                p->multi = NULL;
            } else p->multi = multi;                              /* (bwa_approx_mapQ's value is unused, :345) */
            continue;
        }
        if (p->type == BWA_TYPE_UNIQUE || p->type == BWA_TYPE_REPEAT) {   /* bwa_cal_pac_pos_core */
            const int max_diff = fnr > 0.0 ? bwa_cal_maxdiff(p->len, BWA_AVG_ERR, fnr) : max_mm;
            p->seQ = p->mapQ = bwa_approx_mapQ(p, max_diff);
            put_pos(res + 4 * q++, &p->seq_id, &p->ori_pos, &p->occ_pos);
            p->seQ = p->mapQ = bwa_approx_mapQ(p, max_diff);
        }
        int m = 0;                                                /* bwtse.c:360-366 */
        for (int j = 0; j < p->n_multi; ++j) {
            bwt_multi1_t *r = p->multi + j;
            put_pos(res + 4 * q++, &r->seq_id, &r->ori_pos, &r->occ_pos);
            if (r->occ_pos != p->occ_pos) p->multi[m++] = *r;
        }
        p->n_multi = m;
    }
    free(idx); free(res);
}
