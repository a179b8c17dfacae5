/*
 * san_main.c -- TEST INFRASTRUCTURE ONLY: drives the drop-in host C (bwtaln_gpu.c,
 * bwtgap_gpu.c) the way a host HSA aln does, with the core answered by the CPU
 * restatement (san_core.c), under ASan/UBSan (tests/test_sanitize.py).
 *
 *   san_main <index prefix> <reads.bin> <opt.bin> <batch> <out.bin>
 *
 * reads.bin: u32 n, n u32 lengths, the read codes; opt.bin: one gap_opt_t.
 * Every batch goes through bwa_cal_sa_reg_gap (bwtaln.c:246); out.bin receives per
 * read int32 n_aln then n_aln bwt_aln1_t.  The bwt_splice_match below stands in for
 * the host's splice path (bwtgap.c:748): it makes the first seed call the way
 * bwt_splice_match does (bwtgap.c:797-812) through the drop-in bwt_match_gap, which
 * must answer it from the prefetched table; then it checks bwt_match_gap_batch on
 * several calls against one-at-a-time bwt_match_gap.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../hsa_amd/csrc/bwtaln_gpu.h"
#include "../../include/hsa_bwtaln.h"

static int g_fail = 0;
static long g_splice_calls = 0, g_memo_hits = 0;

static void *read_file(const char *path, size_t *n)
{
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(*n + 16);
    if (fread(p, 1, *n, f) != *n) { perror(path); exit(2); }
    fclose(f);
    return p;
}

/* .bwt: inverseSa0, C[1..4], then ceil(T/16) code words (BWT.c:156-181) */
static BWT *load_bwt(const char *path)
{
    size_t n = 0;
    uint32_t *w = (uint32_t *)read_file(path, &n);
    BWT *b = (BWT *)calloc(1, sizeof(BWT));
    b->inverseSa0 = w[0];
    b->cumulativeFreq = (unsigned *)calloc(5, sizeof(unsigned));
    for (int c = 0; c < 4; ++c) b->cumulativeFreq[c + 1] = w[1 + c];
    b->textLength = w[4];
    const size_t nw = ((size_t)b->textLength + 15) / 16;
    b->bwtCode = (unsigned *)malloc(nw * 4 + 4);
    memcpy(b->bwtCode, w + 5, nw * 4);
    free(w);
    return b;
}

static void free_bwt(BWT *b)
{
    free(b->cumulativeFreq); free(b->bwtCode); free(b);
}

/* the widths bwt_splice_match computes for a seed: bwt_cal_width of the read prefix
 * (bwtgap.c:807), here through the core's width primitive */
static bwt_width_t *prefix_widths(const Idx2BWT *bi, const ubyte_t *seq, int la)
{
    uint64_t off = 0;
    uint32_t len = (uint32_t)la;
    bwt_width_t *w = (bwt_width_t *)calloc((size_t)la + 1, sizeof(bwt_width_t));
    if (hsa_width_batch(hsa_gpu_index_of(bi), 1, &off, &len, seq, (size_t)la, (uint32_t *)w)) g_fail = 1;
    return w;
}

bwt_aln1_t *bwt_splice_match(bwt_aux_t *aux, int *n_aln)
{
    ++g_splice_calls;
    const int L = aux->len, sl = L / 3;
    *n_aln = 0;
    if (sl < 1) return (bwt_aln1_t *)calloc(1, sizeof(bwt_aln1_t));
    /* seed 0 of strand 0 as bwtgap.c:797-812 sets it up */
    bwt_aux_t x = *aux;
    gap_opt_t o = *aux->opt;
    o.mode &= ~BWA_MODE_GAPE;
    o.max_gapo = 0; o.max_gape = 0;
    o.max_diff = aux->opt->max_seed_diff;
    o.seed_len = sl;
    x.opt = &o; x.len = sl; x.strand = 0;
    x.width_back = x.width_seed = prefix_widths(aux->bi_bwt, aux->seq, sl);
    int n = 0;
    uint64_t mh = 0, mm = 0;
    hsa_splice_memo_stats(&mh, &mm);                 /* reset: earlier calls' misses */
    bwt_aln1_t *h = bwt_match_gap(&x, &n);
    hsa_splice_memo_stats(&mh, &mm);
    g_memo_hits += (long)mh;
    if (mh != 1 || mm != 0) { fprintf(stderr, "san: seed call not answered from the prefetch table\n"); g_fail = 1; }
    /* the same call again, alone, after the table: widths reset */
    free(x.width_back);
    x.width_back = x.width_seed = prefix_widths(aux->bi_bwt, aux->seq, sl);
    /* a batch of three differing calls vs the same calls one at a time */
    bwt_aux_t c[3];
    gap_opt_t co[3];
    bwt_width_t *wb[3], *wb1[3];
    bwt_aux_t *cp[3];
    bwt_aln1_t *bo[3];
    int bn[3];
    for (int k = 0; k < 3; ++k) {
        c[k] = *aux;
        co[k] = *aux->opt;
        co[k].seed_len = L;
        c[k].opt = &co[k];
        c[k].strand = k == 1;
        wb[k] = prefix_widths(aux->bi_bwt, k == 1 ? aux->rc_seq : aux->seq, L);
        wb1[k] = (bwt_width_t *)malloc(sizeof(bwt_width_t) * ((size_t)L + 1));
        memcpy(wb1[k], wb[k], sizeof(bwt_width_t) * ((size_t)L + 1));
        c[k].width_back = wb[k];
        c[k].width_seed = k == 0 ? NULL : k == 1 ? wb[k] : wb1[k];   /* NULL, aliased, own */
        cp[k] = &c[k];
    }
    bwt_match_gap_batch(cp, 3, bo, bn);
    for (int k = 0; k < 3; ++k) {
        bwt_aux_t y = c[k];
        bwt_width_t *w2 = prefix_widths(aux->bi_bwt, k == 1 ? aux->rc_seq : aux->seq, L);
        y.width_back = w2;
        y.width_seed = k == 0 ? NULL : k == 1 ? w2 : wb1[k];
        int n1 = 0;
        bwt_aln1_t *one = bwt_match_gap(&y, &n1);
        if (n1 != bn[k] || (n1 > 0 && memcmp(one, bo[k], sizeof(bwt_aln1_t) * (size_t)n1)) ||
            memcmp(w2, wb[k], sizeof(bwt_width_t) * ((size_t)L + 1))) {
            fprintf(stderr, "san: bwt_match_gap_batch call %d differs from bwt_match_gap\n", k);
            g_fail = 1;
        }
        free(one); free(w2); free(bo[k]); free(wb[k]); free(wb1[k]);
    }
    free(x.width_back);
    *n_aln = n;
    return h;
}

int main(int argc, char **argv)
{
    if (argc != 6) { fprintf(stderr, "usage: san_main prefix reads.bin opt.bin batch out.bin\n"); return 2; }
    char path[4096];
    snprintf(path, sizeof path, "%s.index.bwt", argv[1]);
    BWT *f = load_bwt(path);
    snprintf(path, sizeof path, "%s.index.rev.bwt", argv[1]);
    BWT *r = load_bwt(path);
    Idx2BWT bi;
    memset(&bi, 0, sizeof bi);
    bi.bwt = f; bi.rev_bwt = r;
    size_t nb = 0, no = 0;
    uint32_t *rb = (uint32_t *)read_file(argv[2], &nb);
    gap_opt_t *opt = (gap_opt_t *)read_file(argv[3], &no);
    if (no != sizeof(gap_opt_t)) { fprintf(stderr, "opt.bin: %zu bytes\n", no); return 2; }
    const int n = (int)rb[0], batch = atoi(argv[4]);
    const uint32_t *lens = rb + 1;
    const uint8_t *codes = (const uint8_t *)(rb + 1 + n);
    FILE *out = fopen(argv[5], "wb");
    if (!out) { perror(argv[5]); return 2; }
    if (hsa_gpu_attach(&bi)) { fprintf(stderr, "attach failed\n"); return 1; }
    size_t off = 0;
    for (int b0 = 0; b0 < n; b0 += batch) {
        const int m = n - b0 < batch ? n - b0 : batch;
        bwa_seq_t *seqs = (bwa_seq_t *)calloc((size_t)m, sizeof(bwa_seq_t));
        for (int i = 0; i < m; ++i) {
            seqs[i].len = lens[b0 + i];
            seqs[i].seq = (ubyte_t *)malloc(lens[b0 + i] + 1);
            memcpy(seqs[i].seq, codes + off, lens[b0 + i]);
            off += lens[b0 + i];
        }
        bwa_cal_sa_reg_gap(0, &bi, m, seqs, opt, NULL);
        for (int i = 0; i < m; ++i) {
            const int32_t na = seqs[i].n_aln;
            fwrite(&na, 4, 1, out);
            if (na > 0) fwrite(seqs[i].aln, sizeof(bwt_aln1_t), (size_t)na, out);
            free(seqs[i].aln); free(seqs[i].seq);
        }
        free(seqs);
    }
    fclose(out);
    hsa_gpu_detach(&bi);
    free_bwt(f); free_bwt(r); free(rb); free(opt);
    fprintf(stderr, "san: %d reads, %ld splice calls, %ld answered from the prefetch table\n", n, g_splice_calls,
            g_memo_hits);
    return g_fail;
}
