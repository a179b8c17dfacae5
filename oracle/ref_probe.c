/*
 * ref_probe -- drives the COMPILED REFERENCE (oracle/_ref, built by ref.mk from
 * /root/reference) to produce golden vectors.  Test infrastructure only: it is
 * never linked into, loaded by, or called from the product library.
 *
 *   ref_probe aln   <prefix> <reads.bin> <out.bin> [-n X] [-o N] [-e N] [-l N] [-k N]
 *                   [-R N] [-m N] [-M N] [-O N] [-E N] [-d N] [-i N] [-L] [-N] [-B batch] [-G]
 *       Runs bwa_cal_sa_reg_gap (bwtaln.c:246) batch by batch, 100 000 reads per
 *       batch exactly as bwa_aln_core does (bwtaln.c:477, :506), with the options
 *       parsed the way bwa_aln parses them (bwtaln.c:539-575).
 *       out.bin: u32 'HSAH', u32 n; per read: i32 n_aln, u32 flags
 *       (bit0 = bwt_splice_match was called for it), then n_aln raw bwt_aln1_t.
 *   ref_probe occ   <prefix> <pos.bin> <out.bin>
 *       BWTAllOccValue (BWT.c:793) on the forward and reverse BWT at each position,
 *       plus BWTOccValue (BWT.c:682) per character as a cross-check.
 *   ref_probe step  <prefix> <in.bin> <out.bin>
 *       BWTAllSARangesBackward_Bidirection (2BWT-Interface.c:235) on (k,l,rk,rl).
 *   ref_probe width <prefix> <reads.bin> <out.bin>
 *       bwt_cal_width(type=1) (bwtaln.c:73) of every read: (len+1) x {u32 w, i32 bid}.
 *   ref_probe width <prefix> <reads.bin> <out.bin> 0
 *       the same with type 0 (backward; entry 0 is never written: stays 0 from calloc).
 *   ref_probe sa    <prefix> <idx.bin> <out.bin>
 *       BWTSaValue (BWT.c:1195) and BWTRetrievePositionFromSAIndex
 *       (2BWT-Interface.c:329) of each SA index: u32 sa, i32 seqId, u32 ori_pos,
 *       u32 occ_pos per index (seqId / ori_pos preset to -1: left untouched when
 *       the block search finds nothing).
 *   ref_probe meta  <prefix>
 *       prints textLength, inverseSa0, C[0..4] of both BWTs and saInterval.
 *   ref_probe mkfmv <in.bwt> <out.fmv>
 *       the .fmv (occValue + occValueMajor) of a .bwt file, by the reference's own
 *       BWTGenerateOccValueFromBwt (BWTConstruct.c:997) and the occ half of
 *       BWTSaveBwtCodeAndOcc's format (BWTConstruct.c:1209-1240): how bench.py turns a
 *       device-built BWT into index files the reference's BWTLoad reads.
 *
 * reads.bin: u32 n, u32 len[n], then the concatenated 0..4 codes.
 *
 * Built a second time as ref_probe_gpu (-DHSA_GPU_PROBE, oracle/ref.mk): the same driver
 * linked like HSA_gpu_all, i.e. the reference's objects with every drop-in entry point
 * replaced by ours (bwa_cal_sa_reg_gap, bwt_match_gap, the splice path's extensions,
 * widths and SA lookups) and the reference's own bwt_splice_match in between.  Its `aln`
 * times the drop-in end to end on bwa_seq_t batches, splice fallback included, and
 * writes the same out.bin, so the two outputs can be compared read for read (bit 0 of
 * flags is not recorded there).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <sys/time.h>
#include "bwtaln.h"
#include "bwtgap.h"
#include "BWTConstruct.h"
#include "DNACount.h"

static double now_s(void) { struct timeval tv; gettimeofday(&tv, 0); return tv.tv_sec + tv.tv_usec * 1e-6; }

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

typedef struct { uint32_t n; uint32_t *len; uint8_t **seq; } reads_t;

static reads_t load_reads(const char *fn)
{
    size_t sz; uint8_t *buf = slurp(fn, &sz);
    reads_t r; memcpy(&r.n, buf, 4);
    r.len = (uint32_t *)malloc(sizeof(uint32_t) * (r.n + 1));
    memcpy(r.len, buf + 4, 4 * (size_t)r.n);
    r.seq = (uint8_t **)malloc(sizeof(uint8_t *) * (r.n + 1));
    size_t off = 4 + 4 * (size_t)r.n;
    for (uint32_t i = 0; i < r.n; ++i) { r.seq[i] = buf + off; off += r.len[i]; }
    return r;
}

static Idx2BWT *load_index(const char *prefix)
{
    char *str = (char *)calloc(strlen(prefix) + 16, 1);
    strcpy(str, prefix); strcat(str, ".index");
    Idx2BWT *b = BWTLoad2BWT(str, ".sa");
    free(str);
    return b;
}

static bwa_seq_t *g_seqs; static int g_nseqs; static int g_cursor; static uint32_t *g_flags;
#ifdef HSA_GPU_PROBE
int hsa_gpu_attach(const Idx2BWT *bi);      /* the drop-in's upload hook (include/hsa_bwtaln.h) */
#else
/* --wrap=bwt_splice_match: record the read the batch driver is on. */
bwt_aln1_t *__real_bwt_splice_match(bwt_aux_t *aux, int *n);
bwt_aln1_t *__wrap_bwt_splice_match(bwt_aux_t *aux, int *n)
{
    for (; g_cursor < g_nseqs; ++g_cursor)
        if (g_seqs[g_cursor].seq == aux->seq) { g_flags[g_cursor] |= 1; break; }
    return __real_bwt_splice_match(aux, n);
}
#endif

static int cmd_aln(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: aln prefix reads.bin out.bin [opts]\n"); return 1; }
    gap_opt_t *opt = gap_init_opt();
    int opte = -1, batch = 0x186A0, steady = 0;
    for (int a = 4; a < argc; ++a) {
        const char *o = argv[a];
        const char *v = (a + 1 < argc) ? argv[a + 1] : "0";
        if (!strcmp(o, "-n")) { if (strstr(v, ".")) opt->fnr = atof(v), opt->max_diff = -1; else opt->max_diff = atoi(v), opt->fnr = -1.0; ++a; }
        else if (!strcmp(o, "-o")) opt->max_gapo = atoi(v), ++a;
        else if (!strcmp(o, "-e")) opte = atoi(v), ++a;
        else if (!strcmp(o, "-M")) opt->s_mm = atoi(v), ++a;
        else if (!strcmp(o, "-O")) opt->s_gapo = atoi(v), ++a;
        else if (!strcmp(o, "-E")) opt->s_gape = atoi(v), ++a;
        else if (!strcmp(o, "-d")) opt->max_del_occ = atoi(v), ++a;
        else if (!strcmp(o, "-i")) opt->indel_end_skip = atoi(v), ++a;
        else if (!strcmp(o, "-l")) opt->seed_len = atoi(v), ++a;
        else if (!strcmp(o, "-k")) opt->max_seed_diff = atoi(v), ++a;
        else if (!strcmp(o, "-m")) opt->max_entries = atoi(v), ++a;
        else if (!strcmp(o, "-R")) opt->max_top2 = atoi(v), ++a;
        else if (!strcmp(o, "-B")) batch = atoi(v), ++a;   /* probe-only: batch size */
        else if (!strcmp(o, "-L")) opt->mode |= BWA_MODE_LOGGAP;
        else if (!strcmp(o, "-N")) opt->mode |= BWA_MODE_NONSTOP, opt->max_top2 = 0x7fffffff;
        else if (!strcmp(o, "-G")) steady = 1;             /* probe-only: see below */
        else { fprintf(stderr, "unknown option %s\n", o); return 1; }
    }
    if (opte > 0) { opt->max_gape = opte; opt->mode &= ~BWA_MODE_GAPE; }
    /* -G: start in the steady state every batch after a process's first one runs in:
     * bwa_cal_sa_reg_gap clears GAPE in the caller's block through aux->opt (bwtaln.c:261),
     * so from the second batch on local_opt (:254) has it cleared too.
     * bench.py's timed batches are such batches. */
    if (steady) opt->mode &= ~BWA_MODE_GAPE;

    Idx2BWT *bi = load_index(argv[1]);
    bwt_array_t *arr = bwt_array_init();
    reads_t r = load_reads(argv[2]);
#ifdef HSA_GPU_PROBE
    {   /* the index upload (hook after BWTLoad2BWT, bwtaln.c:467) stays outside the timing */
        const double ta = now_s();
        const int rc = hsa_gpu_attach(bi);
        if (rc) { fprintf(stderr, "hsa_gpu_attach failed (%d)\n", rc); return 1; }
        fprintf(stderr, "[ref_probe_gpu] index attached in %.3f s\n", now_s() - ta);
    }
#endif
    FILE *out = fopen(argv[3], "wb");
    uint32_t magic = 0x48415348u; fwrite(&magic, 4, 1, out); fwrite(&r.n, 4, 1, out);
    double t_search = 0;
    for (uint32_t b0 = 0; b0 < r.n; b0 += batch) {
        int n = (int)((r.n - b0) < (uint32_t)batch ? (r.n - b0) : (uint32_t)batch);
        bwa_seq_t *seqs = (bwa_seq_t *)calloc(n, sizeof(bwa_seq_t));
        uint32_t *flags = (uint32_t *)calloc(n, sizeof(uint32_t));
        for (int i = 0; i < n; ++i) {
            bwa_seq_t *p = seqs + i;
            uint32_t L = r.len[b0 + i];
            p->tid = -1;
            p->full_len = p->clip_len = p->len = L;
            p->seq = (ubyte_t *)calloc(L ? L : 1, 1);
            memcpy(p->seq, r.seq[b0 + i], L);
        }
        g_seqs = seqs; g_nseqs = n; g_cursor = 0; g_flags = flags;
        double t0 = now_s();
        bwa_cal_sa_reg_gap(0, bi, n, seqs, opt, arr);
        t_search += now_s() - t0;
        for (int i = 0; i < n; ++i) {
            bwa_seq_t *p = seqs + i;
            int32_t na = p->n_aln;
            fwrite(&na, 4, 1, out); fwrite(&flags[i], 4, 1, out);
            if (na > 0) fwrite(p->aln, sizeof(bwt_aln1_t), na, out);
            free(p->aln); free(p->seq);
        }
        free(seqs); free(flags);
    }
    fclose(out);
    fprintf(stderr, "[ref_probe%s] bwa_cal_sa_reg_gap: %u reads in %.3f s (%.1f reads/s)\n",
#ifdef HSA_GPU_PROBE
            "_gpu",
#else
            "",
#endif
            r.n, t_search, t_search > 0 ? r.n / t_search : 0.0);
    printf("%.6f\n", t_search);
    return 0;
}

static int cmd_occ(int argc, char **argv)
{
    Idx2BWT *bi = load_index(argv[1]);
    size_t sz; uint32_t *in = (uint32_t *)slurp(argv[2], &sz);
    uint32_t n = in[0];
    FILE *out = fopen(argv[3], "wb");
    BWT *bw[2] = { bi->bwt, bi->rev_bwt };
    for (int d = 0; d < 2; ++d)
        for (uint32_t i = 0; i < n; ++i) {
            unsigned int ALIGN_16 occ[4];
            uint32_t o2[4];
            BWTAllOccValue(bw[d], in[1 + i], occ);
            for (int c = 0; c < 4; ++c) {
                o2[c] = BWTOccValue(bw[d], in[1 + i], c);
                if (o2[c] != occ[c]) { fprintf(stderr, "BWTOccValue/BWTAllOccValue disagree at %u\n", in[1 + i]); return 2; }
            }
            fwrite(occ, 4, 4, out);
        }
    fclose(out);
    return 0;
}

static int cmd_step(int argc, char **argv)
{
    Idx2BWT *bi = load_index(argv[1]);
    size_t sz; uint32_t *in = (uint32_t *)slurp(argv[2], &sz);
    uint32_t n = in[0];
    FILE *out = fopen(argv[3], "wb");
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t *q = in + 1 + 4 * (size_t)i;
        unsigned int k[4], l[4], rk[4], rl[4];
        BWTAllSARangesBackward_Bidirection(bi, q[0], q[1], q[2], q[3], k, l, rk, rl);
        fwrite(k, 4, 4, out); fwrite(l, 4, 4, out); fwrite(rk, 4, 4, out); fwrite(rl, 4, 4, out);
    }
    fclose(out);
    return 0;
}

static int cmd_width(int argc, char **argv)
{
    Idx2BWT *bi = load_index(argv[1]);
    reads_t r = load_reads(argv[2]);
    FILE *out = fopen(argv[3], "wb");
    for (uint32_t i = 0; i < r.n; ++i) {
        bwt_width_t *w = (bwt_width_t *)calloc(r.len[i] + 1, sizeof(bwt_width_t));
        bwt_cal_width(bi, (int)r.len[i], r.seq[i], w, argc > 4 ? atoi(argv[4]) : 1);
        fwrite(w, sizeof(bwt_width_t), r.len[i] + 1, out);
        free(w);
    }
    fclose(out);
    return 0;
}

static int cmd_sa(int argc, char **argv)
{
    Idx2BWT *bi = load_index(argv[1]);
    size_t sz; uint32_t *in = (uint32_t *)slurp(argv[2], &sz);
    uint32_t n = in[0];
    FILE *out = fopen(argv[3], "wb");
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t idx = in[1 + i];
        uint32_t v[4];
        v[0] = BWTSaValue(bi->bwt, idx);
        unsigned int sid = 0xffffffffu, ori = 0xffffffffu, occ = 0;
        BWTRetrievePositionFromSAIndex(bi, idx, &sid, &ori, &occ);
        v[1] = sid; v[2] = ori; v[3] = occ;
        fwrite(v, 4, 4, out);
    }
    fclose(out);
    return 0;
}

static int cmd_meta(int argc, char **argv)
{
    Idx2BWT *bi = load_index(argv[1]);
    BWT *bw[2] = { bi->bwt, bi->rev_bwt };
    for (int d = 0; d < 2; ++d)
        printf("%s T=%u isa0=%u C=%u,%u,%u,%u,%u saInterval=%u\n", d ? "rev" : "fwd",
               bw[d]->textLength, bw[d]->inverseSa0, bw[d]->cumulativeFreq[0], bw[d]->cumulativeFreq[1],
               bw[d]->cumulativeFreq[2], bw[d]->cumulativeFreq[3], bw[d]->cumulativeFreq[4], bw[d]->saInterval);
    printf("sizeof bwt_aln1_t=%zu gap_opt_t=%zu bwa_seq_t=%zu bwt_aux_t=%zu BWT=%zu Idx2BWT=%zu HSP=%zu\n",
           sizeof(bwt_aln1_t), sizeof(gap_opt_t), sizeof(bwa_seq_t), sizeof(bwt_aux_t), sizeof(BWT),
           sizeof(Idx2BWT), sizeof(HSP));
    return 0;
}

static int cmd_mkfmv(int argc, char **argv)
{
    if (argc < 3) { fprintf(stderr, "usage: mkfmv in.bwt out.fmv\n"); return 1; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", argv[1]); return 1; }
    unsigned int cf[ALPHABET_SIZE + 1] = {0}, isa0 = 0;
    if (fread(&isa0, 4, 1, f) != 1 || fread(cf + 1, 4, ALPHABET_SIZE, f) != ALPHABET_SIZE) { fprintf(stderr, "short .bwt\n"); return 1; }
    BWT b;
    memset(&b, 0, sizeof b);
    b.textLength = cf[ALPHABET_SIZE];
    b.inverseSa0 = isa0;
    b.cumulativeFreq = cf;
    b.bwtSizeInWord = BWTResidentSizeInWord(b.textLength) + WORD_BETWEEN_OCC / 2;      /* as BWTLoad, BWT.c:176 */
    b.bwtCode = (unsigned int *)calloc(b.bwtSizeInWord, 4);
    const unsigned int nw = BWTFileSizeInWord(b.textLength);
    if (fread(b.bwtCode, 4, nw, f) != nw) { fprintf(stderr, "short .bwt codes\n"); return 1; }
    fclose(f);
    BWTClearTrailingBwtCode(&b);
    b.occSizeInWord = BWTOccValueMinorSizeInWord(b.textLength);
    b.occMajorSizeInWord = BWTOccValueMajorSizeInWord(b.textLength);
    b.occValue = (unsigned int *)calloc(b.occSizeInWord, 4);
    b.occValueMajor = (unsigned int *)calloc(b.occMajorSizeInWord, 4);
    unsigned int *dt = (unsigned int *)malloc(DNA_OCC_CNT_TABLE_SIZE_IN_WORD * sizeof(unsigned int));
    GenerateDNAOccCountTable(dt);
    BWTGenerateOccValueFromBwt(b.bwtCode, b.occValue, b.occValueMajor, b.textLength, dt);
    FILE *o = fopen(argv[2], "wb");
    if (!o) { fprintf(stderr, "cannot write %s\n", argv[2]); return 1; }
    fwrite(&b.inverseSa0, 4, 1, o);
    fwrite(cf + 1, 4, ALPHABET_SIZE, o);
    fwrite(b.occValue, 4, b.occSizeInWord, o);
    fwrite(b.occValueMajor, 4, b.occMajorSizeInWord, o);
    fclose(o);
    free(b.bwtCode); free(b.occValue); free(b.occValueMajor); free(dt);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 3) { fprintf(stderr, "usage: ref_probe aln|occ|step|width|meta ...\n"); return 1; }
    if (!strcmp(argv[1], "aln")) return cmd_aln(argc - 1, argv + 1);
    if (!strcmp(argv[1], "occ")) return cmd_occ(argc - 1, argv + 1);
    if (!strcmp(argv[1], "step")) return cmd_step(argc - 1, argv + 1);
    if (!strcmp(argv[1], "width")) return cmd_width(argc - 1, argv + 1);
    if (!strcmp(argv[1], "meta")) return cmd_meta(argc - 1, argv + 1);
    if (!strcmp(argv[1], "sa")) return cmd_sa(argc - 1, argv + 1);
    if (!strcmp(argv[1], "mkfmv")) return cmd_mkfmv(argc - 1, argv + 1);
    fprintf(stderr, "unknown command %s\n", argv[1]);
    return 1;
}
