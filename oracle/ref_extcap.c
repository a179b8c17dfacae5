/*
 * ref_extcap -- records every seed extension the COMPILED REFERENCE makes in its
 * splice path: the calls of bwt_splice_match (bwtgap.c:748) to bwt_extend_foreward /
 * bwt_extend_backward (bwtgap.c:640-663: gap_reset_stack + the seed's entry +
 * bwt_backtracing_search, :346-511), inputs and outputs.  Test infrastructure only
 * (golden vectors for the extension search); never linked into, loaded
 * by, or called from the product library.
 *
 *   ref_extcap <prefix> <reads.bin> <out.bin> [-n X] [-o N] [-e N] [-k N] [-l N] [-B batch]
 *
 * Link recipe (ref.mk, target ref_extcap): the reference's bwtgap.o enters twice --
 *   bwtgap_weakx.o  bwt_extend_foreward / bwt_extend_backward weakened, so
 *                   bwt_splice_match's calls (through the PLT under -fPIC) reach the
 *                   recorder below;
 *   bwtgap_renx.o   both renamed (ref_bwt_extend_*) and every other global made local:
 *                   the unmodified reference code the recorder calls.
 *
 * A call reads the strand sequence and the widths (width_back backward, width_fore
 * forward; only .bid) inside one window of read positions, from the caller's
 * arguments alone (the extension length len = aux->len, aln->start / aln->end and the
 * bound *max_pos):
 *   backward: positions [min(start - len, max_pos), max(start, max_pos + 1)]
 *   forward:  positions [min(end, max_pos - 1), max(end + len, max_pos)]
 * (bwtgap.c:392, :425, :439-446, 2BWT-Interface.c:394-439); empty for a negative
 * length (see record()).  The window is recorded
 * (sequence bytes outside [start - len, start - 1] / [end + 1, end + len], which the
 * search never reads, recorded as 0xFF), and the restatement reads nothing outside it.
 *
 * out.bin: u32 'EXCP', then one record per call:
 *   i32 dir (1 backward, 0 forward), len, strand, n_stacks, max_pos_in, lo, n, read_len
 *   gap_opt_t opt (64 B, as the call sees it)
 *   bwt_aln1_t aln_in
 *   u8  seq[n]   strand sequence at positions lo .. lo + n - 1
 *   i32 bid[n]   the direction's width[].bid at the same positions
 *   i32 ret, max_pos_out
 *   bwt_aln1_t aln_out
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "bwtaln.h"
#include "bwtgap.h"

int ref_bwt_extend_foreward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_right);
int ref_bwt_extend_backward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_left);

static FILE *g_out;
static long g_calls;

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

static int record(bwt_aux_t *aux, bwt_aln1_t *aln, int *mp, int dir)
{
    const int len = aux->len, L = aux->max_len;    /* fixed-length read sets: max_len = L */
    int lo, hi;
    if (dir) { lo = imin(aln->start - len, *mp); hi = imax(aln->start, *mp + 1); }
    else { lo = imin(aln->end, *mp - 1); hi = imax(aln->end + len, *mp); }
    /* a negative length (the splice path makes such calls) gives the seed's entry a
     * score field of 2047 (info = score << 21 | i with i < 0), so the search stops at its
     * first pop unless NONSTOP: nothing is read */
    if (len < 0 && !(aux->opt->mode & BWA_MODE_NONSTOP)) lo = 0, hi = -1;
    else if (len < 0 || lo < 0 || hi > L) {
        fprintf(stderr, "ref_extcap: call outside the read (len %d, window [%d, %d], read %d)\n", len, lo, hi, L);
        exit(2);
    }
    const int n = hi - lo + 1;
    const ubyte_t *seq = aux->strand == 0 ? aux->seq : aux->rc_seq;
    const bwt_width_t *w = dir ? aux->width_back : aux->width_fore;
    int32_t hdr[8] = {dir, len, aux->strand, aux->stack->n_stacks, *mp, lo, n, L};
    fwrite(hdr, 4, 8, g_out);
    fwrite(aux->opt, sizeof(gap_opt_t), 1, g_out);
    fwrite(aln, sizeof(bwt_aln1_t), 1, g_out);
    /* the sequence is read at [start - len, start - 1] (backward) or [end + 1, end + len]
     * (forward) only; other window positions are recorded as 0xFF */
    const int s0 = dir ? aln->start - len : aln->end + 1, s1 = dir ? aln->start - 1 : aln->end + len;
    (void)L;
    for (int p = lo; p <= hi; ++p) {
        const uint8_t c = p >= s0 && p <= s1 ? seq[p] : 0xFF;
        fwrite(&c, 1, 1, g_out);
    }
    for (int p = lo; p <= hi; ++p) fwrite(&w[p].bid, 4, 1, g_out);
    const int ret = dir ? ref_bwt_extend_backward(aux, aln, mp) : ref_bwt_extend_foreward(aux, aln, mp);
    int32_t tail[2] = {ret, *mp};
    fwrite(tail, 4, 2, g_out);
    fwrite(aln, sizeof(bwt_aln1_t), 1, g_out);
    ++g_calls;
    return ret;
}

int bwt_extend_foreward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_right) { return record(aux, aln, _right, 0); }
int bwt_extend_backward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_left) { return record(aux, aln, _left, 1); }

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
    if (argc < 4) { fprintf(stderr, "usage: ref_extcap prefix reads.bin out.bin [opts]\n"); return 1; }
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
    uint32_t magic = 0x50435845u; fwrite(&magic, 4, 1, g_out);
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
    fprintf(stderr, "[ref_extcap] %ld extension calls recorded\n", g_calls);
    return 0;
}
