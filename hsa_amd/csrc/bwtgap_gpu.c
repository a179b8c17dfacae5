/*
 * bwtgap_gpu.c -- host side of the drop-in bwt_match_gap (bwtgap.c:118-331, declared
 * bwtgap.h:26) on the MI355X search core: the calls the host's splice path makes
 * (bwt_splice_match's seed and anchor searches, bwtgap.c:812, :919, :1192), with the
 * caller's widths, width_seed NULL or aliased, and width_back handed back as
 * gap_shadow leaves it.  Its own object so that a host can take the GPU
 * bwa_cal_sa_reg_gap alone (bwtaln_gpu.o) or both entry points.
 */
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

/* bwt_match_gap (bwtgap.c:118, declared bwtgap.h:26): the reference's entry point,
 * one call at a time (a batch of one).  Same return contract: a calloc'd array,
 * never NULL, freed by the caller with free(). */
bwt_aln1_t *bwt_match_gap(bwt_aux_t *aux, int *_n_aln)
{
    bwt_aln1_t *out = NULL;
    bwt_match_gap_batch(&aux, 1, &out, _n_aln);
    return out;
}

