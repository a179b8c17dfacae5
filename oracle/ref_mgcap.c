/*
 * ref_mgcap -- records every bwt_match_gap call the COMPILED REFERENCE makes while
 * its bwa_cal_sa_reg_gap runs over a read set: the main-path calls (bwtaln.c:350)
 * and the splice path's seed and anchor calls (bwtgap.c:812, :919, :1192).  Test
 * infrastructure only (golden vectors for the caller-width search);
 * never linked into, loaded by, or called from the product library.
 *
 *   ref_mgcap <prefix> <reads.bin> <out.bin> [-n X] [-o N] [-e N] [-k N] [-l N] [-B batch]
 *
 * Link recipe (ref.mk, target ref_mgcap): the reference's bwtgap.o enters twice --
 *   bwtgap_weak.o  bwt_match_gap weakened, so every call (bwtaln.c's, and
 *                  bwt_splice_match's, which go through the PLT under -fPIC) reaches
 *                  the recorder below;
 *   bwtgap_ren.o   the definition renamed to ref_bwt_match_gap and every other global
 *                  made local: the unmodified reference code the recorder calls.
 *
 * out.bin: u32 'MGCP', then one record per call:
 *   i32 strand, len, seed (0 width_seed NULL, 1 own array, 2 aliased to width_back),
 *       n_stacks (aux->stack), n_seed (entries of width_seed recorded)
 *   gap_opt_t opt (64 B, as the call sees it)
 *   u8  seq[len]                       the searched sequence (strand ? rc_seq : seq)
 *   bwt_width_t width_back[len + 1]    before the call
 *   bwt_width_t width_seed[n_seed]     seed == 1 only
 *   i32 n_aln, bwt_aln1_t hits[n_aln]
 *   bwt_width_t width_back[len + 1]    after the call (gap_shadow, bwtgap.c:94-105)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "bwtaln.h"
#include "bwtgap.h"

bwt_aln1_t *ref_bwt_match_gap(bwt_aux_t *aux, int *n);

static FILE *g_out;
static long g_calls;

bwt_aln1_t *bwt_match_gap(bwt_aux_t *aux, int *n_aln)
{
    const ubyte_t *seq = aux->strand == 1 ? aux->rc_seq : aux->seq;
    int32_t hdr[5];
    hdr[0] = aux->strand;
    hdr[1] = aux->len;
    hdr[2] = aux->width_seed == NULL ? 0 : aux->width_seed == aux->width_back ? 2 : 1;
    hdr[3] = aux->stack->n_stacks;
    hdr[4] = 0;
    if (hdr[2] == 1) {
        int s = aux->opt->seed_len;
        if (s < 0 || s > aux->len) {   /* Q5: the reference reads outside width_seed */
            fprintf(stderr, "ref_mgcap: call with seed_len %d, len %d is undefined in the reference\n", s, aux->len);
            exit(2);
        }
        hdr[4] = s + 1;
    }
    fwrite(hdr, 4, 5, g_out);
    fwrite(aux->opt, sizeof(gap_opt_t), 1, g_out);
    fwrite(seq, 1, (size_t)aux->len, g_out);
    fwrite(aux->width_back, sizeof(bwt_width_t), (size_t)aux->len + 1, g_out);
    if (hdr[2] == 1) fwrite(aux->width_seed, sizeof(bwt_width_t), (size_t)hdr[4], g_out);
    bwt_aln1_t *a = ref_bwt_match_gap(aux, n_aln);
    int32_t na = *n_aln;
    fwrite(&na, 4, 1, g_out);
    if (na > 0) fwrite(a, sizeof(bwt_aln1_t), (size_t)na, g_out);
    fwrite(aux->width_back, sizeof(bwt_width_t), (size_t)aux->len + 1, g_out);
    ++g_calls;
    return a;
}

static void *slurp(const char *fn, size_t *sz)
{
    FILE *f = fopen(fn, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", fn); exit(1); }
    fseek(f, 0, SEEK_END); *sz = (size_t)ftell(f); fseek(f, 0, SEEK_SET);
    void *p = malloc(*sz ? *sz : 1);
    if (*sz && fread(p, 1, *sz, f) != *sz) { fprintf(stderr, "short read %s\n", fn); exit(1); }
    fclose(f);
    return p;
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: ref_mgcap prefix reads.bin out.bin [opts]\n"); return 1; }
    gap_opt_t *opt = gap_init_opt();
    int opte = -1, batch = 0x186A0;
    for (int a = 4; a < argc; ++a) {           /* bwa_aln's flags (bwtaln.c:539-575) */
        const char *o = argv[a];
        const char *v = (a + 1 < argc) ? argv[a + 1] : "0";
        if (!strcmp(o, "-n")) { if (strstr(v, ".")) opt->fnr = atof(v), opt->max_diff = -1; else opt->max_diff = atoi(v), opt->fnr = -1.0; ++a; }
        else if (!strcmp(o, "-o")) opt->max_gapo = atoi(v), ++a;
        else if (!strcmp(o, "-e")) opte = atoi(v), ++a;
        else if (!strcmp(o, "-k")) opt->max_seed_diff = atoi(v), ++a;
        else if (!strcmp(o, "-l")) opt->seed_len = atoi(v), ++a;
        else if (!strcmp(o, "-B")) batch = atoi(v), ++a;
        else { fprintf(stderr, "unknown option %s\n", o); return 1; }
    }
    if (opte > 0) { opt->max_gape = opte; opt->mode &= ~BWA_MODE_GAPE; }

    char *str = (char *)calloc(strlen(argv[1]) + 16, 1);
    strcpy(str, argv[1]); strcat(str, ".index");
    Idx2BWT *bi = BWTLoad2BWT(str, ".sa");
    bwt_array_t *arr = bwt_array_init();
    size_t sz; uint8_t *buf = (uint8_t *)slurp(argv[2], &sz);
    uint32_t n; memcpy(&n, buf, 4);
    const uint32_t *len = (const uint32_t *)(buf + 4);
    size_t off = 4 + 4 * (size_t)n;
    g_out = fopen(argv[3], "wb");
    uint32_t magic = 0x5043474Du; fwrite(&magic, 4, 1, g_out);
    for (uint32_t b0 = 0; b0 < n; b0 += (uint32_t)batch) {
        int m = (int)((n - b0) < (uint32_t)batch ? (n - b0) : (uint32_t)batch);
        bwa_seq_t *seqs = (bwa_seq_t *)calloc(m, sizeof(bwa_seq_t));
        for (int i = 0; i < m; ++i) {
            bwa_seq_t *p = seqs + i;
            uint32_t L = len[b0 + i];
            p->tid = -1;
            p->full_len = p->clip_len = p->len = L;
            p->seq = (ubyte_t *)calloc(L ? L : 1, 1);
            memcpy(p->seq, buf + off, L);
            off += L;
        }
        bwa_cal_sa_reg_gap(0, bi, m, seqs, opt, arr);
        for (int i = 0; i < m; ++i) { free(seqs[i].aln); free(seqs[i].seq); }
        free(seqs);
    }
    fclose(g_out);
    fprintf(stderr, "[ref_mgcap] %ld bwt_match_gap calls recorded\n", g_calls);
    return 0;
}
