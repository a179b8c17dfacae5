/*
 * bwtse_gpu.c -- host side of the drop-in bwa_cal_pac_pos (bwtse.c:350-369): the SAM
 * stage's SA -> position step with the SA lookups batched on the GPU.
 *
 * The reference walks each read and calls BWTRetrievePositionFromSAIndex
 * (2BWT-Interface.c:329) once for its SA value (bwa_cal_pac_pos_core, bwtse.c:139-148)
 * and once per extra hit position (bwtse.c:359-365): up to saInterval - 1 dependent
 * rank queries each (BWTSaValue, BWT.c:1195).  Here those lookups are gathered in the
 * order the reference makes them, answered by one hsa_sa_position_batch launch
 * (k_sa_position, hsa_sa.hip), and written back with the same per-read updates in the
 * same order: mapQ before and after the position (the host's bwa_approx_mapQ), seq_id
 * and ori_pos only when a block holds the position, the duplicate-position filter of
 * the extra hits.  Reads of type BWA_TYPE_SPLICING keep the host's
 * bwt_aln2pos_splicing (bwtse.c:295), part of the splice path that stays host code.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hsa_bwtaln.h"
#include "bwtaln_gpu.h"

/* the host's own functions this step calls (bwtse.c:122, bwtaln.c:46, bwtse.c:295) */
#pragma weak bwa_approx_mapQ
#pragma weak bwa_cal_maxdiff
#pragma weak bwt_aln2pos_splicing
extern int bwa_approx_mapQ(const bwa_seq_t *p, int mm);
extern int bwa_cal_maxdiff(int l, double err, double thres);
extern void bwt_aln2pos_splicing(const Idx2BWT *bi_bwt, bwa_seq_t *seq, int max_diff, float fnr);

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

void bwa_cal_pac_pos(const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seq, int max_mm, float fnr)
{
    if (!bwa_approx_mapQ || !bwa_cal_maxdiff || !bwt_aln2pos_splicing) {
        fprintf(stderr, "[bwa_cal_pac_pos] the host lacks bwa_approx_mapQ / bwa_cal_maxdiff / bwt_aln2pos_splicing\n");
        exit(1);
    }
    /* the lookups of bwtse.c:352-366 in the order the reference makes them */
    size_t n = 0;
    for (int i = 0; i < n_seqs; ++i) {
        const bwa_seq_t *p = seq + i;
        if (p->type == BWA_TYPE_SPLICING) continue;
        if (p->type == BWA_TYPE_UNIQUE || p->type == BWA_TYPE_REPEAT) ++n;
        if (p->n_multi > 0) n += (size_t)p->n_multi;
    }
    uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    uint32_t *res = (uint32_t *)malloc(sizeof(uint32_t) * 4 * (n + 1));
    size_t q = 0;
    for (int i = 0; i < n_seqs; ++i) {
        const bwa_seq_t *p = seq + i;
        if (p->type == BWA_TYPE_SPLICING) continue;
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
        if (p->type == BWA_TYPE_SPLICING) {                      /* bwtse.c:356-357 */
            bwt_aln2pos_splicing(bi_bwt, p, max_mm, fnr);
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
