/*
 * hsa_bwtaln.h -- the drop-in boundary: reference-compatible entry points and
 * struct layouts of the HSA `aln` search path, implemented on the MI355X core.
 *
 * Linking libhsa_gpu.so in place of the reference's definitions (see
 * INTEGRATION.md) keeps the host program unchanged:
 *
 *   bwa_cal_sa_reg_gap   replaces bwtaln.c:246  (declared bwtaln.h:199-200)
 *   bwt_match_gap        replaces bwtgap.c:118  (declared bwtgap.h:26)
 *   bwt_match_gap_batch  new: many bwt_match_gap calls in one GPU pass
 *   hsa_gpu_attach       new hook, called once after BWTLoad2BWT (bwtaln.c:467)
 *   hsa_gpu_detach       new hook, before BWTFree2BWT (bwtaln.c:527)
 *   hsa_gpu_set_devices  new hook: device slots one call is split over (see below)
 *   bwa_cal_pac_pos      replaces bwtse.c:350 (SAM stage: SA -> position, batched)
 *   generate_sam_se_core replaces bwtse.c:884 (the SAM stage on host threads)
 *
 * The structs below are declared here only so that the library reads and writes
 * the host's objects at the right offsets; their layouts are those of the
 * reference on x86-64 (sizes checked by static asserts in bwtaln_gpu.c and by
 * tests/test_abi.py against the compiled reference).
 */
#ifndef HSA_BWTALN_H
#define HSA_BWTALN_H
#include <stdint.h>
#include "hsa_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef uint32_t bwtint_t;       /* 2BWT-Interface.h:26 */
typedef unsigned char ubyte_t;

/* BWT.h:61-83 (only textLength, inverseSa0, cumulativeFreq and bwtCode are read) */
typedef struct BWT {
    unsigned int textLength, saInterval, inverseSaInterval, inverseSa0;
    unsigned int *cumulativeFreq, *bwtCode, *occValue, *occValueMajor, *saValue, *inverseSa, *cachedSaIndex;
    unsigned int cachedSaIndexNumOfChar;
    unsigned int *saValueOnBoundary, *decodeTable;
    unsigned int decodeTableGenerated, bwtSizeInWord, occSizeInWord, occMajorSizeInWord, saValueSizeInWord,
                 inverseSaSizeInWord, cachedSaIndexSizeInWord;
} BWT;

/* HSP.h:41-46 and :65-72 (the block table feeds SA -> position) */
typedef struct { int chrID; unsigned int blockStart, blockEnd, ori; } ChrBlock;
typedef struct HSP {
    unsigned int *packedDNA;
    int chrNum;
    char **chrName;
    int numOfBlock;
    ChrBlock *blockList;
    unsigned int dnaLength;
} HSP;
struct MMPool;
/* 2BWT-Interface.h:29-36 */
typedef struct _Idx2BWT {
    struct MMPool *mmPool;
    BWT *bwt, *rev_bwt;
    struct HSP *hsp;
    unsigned char charMap[256], complementMap[256];
} Idx2BWT;

/* bwtaln.h:36-39 */
typedef struct { bwtint_t w; int bid; } bwt_width_t;

/* bwtaln.h:41-50 -- the hit record (36 bytes) */
typedef struct {
    uint32_t n_mm:16, n_gapo:8, n_gape:8;
    bwtint_t k, l;
    bwtint_t rev_k, rev_l;
    bwtint_t type:30, strand:2;
    int start, end;
    int score;
} bwt_aln1_t;

/* bwtaln.h:52-68 -- the reference's stack, allocated here only to hand to the
 * host's bwt_splice_match */
typedef struct {
    uint32_t info;
    uint32_t n_mm:8, n_gapo:8, n_gape:8, state:2, n_seed_mm:6;
    bwtint_t k, l, rev_k, rev_l;
    int last_diff_pos;
} gap_entry_t;
typedef struct { int n_entries, m_entries; gap_entry_t *stack; } gap_stack1_t;
typedef struct { int n_stacks, best, n_entries; gap_stack1_t *stacks; } gap_stack_t;

typedef uint32_t bwa_cigar_t;
/* bwtaln.h:84-91 -- one more hit position of a read (40 bytes) */
typedef struct bwt_multi1_t {
    uint32_t n_cigar:15, gap:8, mm:8, strand:1;
    bwtint_t sa, ori_pos, occ_pos;
    unsigned int seq_id;
    unsigned int aln_id;
    int start, end;
    bwa_cigar_t *cigar;
} bwt_multi1_t;
/* bwtaln.h:93-120 (208 bytes) */
typedef struct {
    char *name;
    ubyte_t *seq, *rseq, *qual;
    uint32_t len:19, strand:1, type:3, dummy:1, extra_flag:8;
    uint32_t n_mm:8, n_gapo:8, n_gape:8, mapQ:8;
    int score;
    int clip_len;
    int n_aln;
    bwt_aln1_t *aln;
    int start, end;
    int n_multi;
    struct bwt_multi1_t *multi;
    bwtint_t sa, ori_pos, occ_pos;
    uint32_t seq_id;
    uint64_t c1:28, c2:28, seQ:8;
    int n_cigar;
    bwa_cigar_t *cigar;
    int tid;
    char bc[64];
    uint32_t full_len:20, nm:12;
    char *md;
} bwa_seq_t;

/* bwtaln.h:122-131 mode bits */
/* bwtaln.h:9-13 */
#define BWA_TYPE_NO_MATCH   0
#define BWA_TYPE_UNIQUE     1
#define BWA_TYPE_REPEAT     2
#define BWA_TYPE_SPLICING   4

#define BWA_MODE_GAPE       0x01
#define BWA_MODE_COMPREAD   0x02
#define BWA_MODE_LOGGAP     0x04
#define BWA_MODE_NONSTOP    0x10

/* bwtaln.h:133-143 (64 bytes) */
typedef struct {
    int s_mm, s_gapo, s_gape;
    int mode;
    int indel_end_skip, max_del_occ, max_entries;
    float fnr;
    int max_diff, max_gapo, max_gape;
    int max_seed_diff, seed_len;
    int n_threads;
    int max_top2;
    int trim_qual;
} gap_opt_t;

struct bwt_array_t;
/* bwtaln.h:156-169 (96 bytes) */
typedef struct _bwt_aux_t {
    Idx2BWT *bi_bwt;
    bwt_width_t *width_back, *width_fore, *width_seed;
    ubyte_t *seq, *rc_seq;
    gap_opt_t *opt;
    gap_stack_t *stack;
    struct bwt_array_t *arr;
    int start, end;
    int strand;
    int len;
    int max_len;
} bwt_aux_t;

/* ---- drop-in entry points (reference ABI) ---- */
void bwa_cal_sa_reg_gap(int tid, const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, const gap_opt_t *opt,
                        struct bwt_array_t *arr);
/* bwt_match_gap: replaces bwtgap.c:118 (declared bwtgap.h:26).  The host's splice path
 * (bwt_splice_match, bwtgap.c:748) calls it with its own widths; the result array is
 * calloc'd (capacity as the reference's, never NULL) and aux->width_back is left as
 * gap_shadow leaves it. */
bwt_aln1_t *bwt_match_gap(bwt_aux_t *aux, int *_n_aln);
/* n independent bwt_match_gap calls in one GPU pass: out[i] / n_out[i] as
 * bwt_match_gap would return them for aux[i] (new entry point). */
int  bwt_match_gap_batch(bwt_aux_t *const *aux, int n, bwt_aln1_t **out, int *n_out);
int  hsa_gpu_attach(const Idx2BWT *bi_bwt);
void hsa_gpu_detach(const Idx2BWT *bi_bwt);
/* bwt_extend_backward / bwt_extend_foreward: replace bwtgap.c:640 / :654 (declared
 * bwtgap.h; -> bwt_backtracing_search :346-511).  Same effects on *aln and the bound.
 * Called from the drop-in bwa_cal_sa_reg_gap's splice runner, a batch's calls run as
 * GPU batches (hsa_extend_batch); called elsewhere, one GPU call each. */
int  bwt_extend_backward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_left);
int  bwt_extend_foreward(bwt_aux_t *aux, bwt_aln1_t *aln, int *_right);
/* bwt_cal_width: replaces bwtaln.c:73 (declared bwtaln.h).  Writes the entries the
 * reference writes (type 1: 0..len, type 0: 1..len) and returns its value; the splice
 * path's calls are answered from a table filled on the GPU per batch. */
int  bwt_cal_width(const Idx2BWT *bi_bwt, int len, const ubyte_t *str, bwt_width_t *width, int type);
/* Device slots: each bwa_cal_sa_reg_gap call splits its reads into n contiguous parts,
 * searched concurrently on slots 0..n-1 (slot k on device k % hsa_device_count(), one
 * host thread and one uploaded index per slot; several slots may share a device).
 * Reads are independent except for the option-regime switch after the first splice
 * fallback read (bwtaln.c:254-363), which the split keeps: regime A is
 * searched over all slots, the first fallback read is found over all of them, and the
 * reads after it are searched again in regime B.  Results are those of one device.
 * 1 <= n <= HSA_MAX_SLOTS; default 1, or the HSA_GPU_DEVICES environment variable.
 * Returns 0, or HSA_E_ARG (n out of range or no device). */
#define HSA_MAX_SLOTS 16
int  hsa_gpu_set_devices(int n);

/* bwa_cal_pac_pos: replaces bwtse.c:350 (declared bwtse.h).  The SAM stage's
 * SA -> position step: the lookups of every non-splicing read of the batch (its SA
 * value bwtse.c:146 and every other hit position bwtse.c:362) run as one GPU batch
 * (hsa_sa_position_batch: BWTSaValue + BWTRetrievePositionFromSAIndex), then the same
 * per-read updates (mapQ, seq_id/ori_pos/occ_pos, duplicate-position filter) in the
 * same order.  A splicing read's lookups (the first 50 rows of both segments,
 * bwtse.c:320) join the same batch, and its segment pairing (bwt_aln2pos_splicing /
 * bwt_combine_segment_splice, bwtse.c:295-348, :197-235) is restated.
 * Needs the host's bwa_approx_mapQ and bwa_cal_maxdiff. */
void bwa_cal_pac_pos(const Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, int max_mm, float fnr);

/* generate_sam_se_core: replaces bwtse.c:884 (declared bwtse.h; called once per batch,
 * bwtaln.c:514).  The SAM stage of one batch on host threads (HSA_SAM_THREADS, default
 * the process's CPUs up to 16): the hit choice of bwt_aln2seq_core with each read's
 * drand48 numbers found by jump-ahead (the process's drand48 state left where the
 * reference leaves it), bwa_cal_pac_pos (whichever the program links: ours runs the
 * lookups on the GPU), the host's bwa_refine_gapped on chunks of reads, and
 * bwa_print_sam1's lines restated into per-chunk buffers written in read order: the
 * reference's bytes.  The first batch checks the restated printing against the host's
 * bwa_print_sam1 and falls back to it if they differ (hsa_amd/csrc/bwtsam_gpu.c). */
void generate_sam_se_core(Idx2BWT *bi_bwt, int n_seqs, bwa_seq_t *seqs, gap_opt_t *opt, int n_occ);

/* The host's splice fallback (bwtgap.c:748).  Weak: when the host program does
 * not provide it, reads without a hit are left with n_aln = 0. */
bwt_aln1_t *bwt_splice_match(bwt_aux_t *aux, int *n_aln) __attribute__((weak));

/* ---- flat form of bwa_cal_sa_reg_gap for bindings (plain arrays) ----
 * Same semantics and the same side effects on *opt.  Per-read flags:
 *   HSA_F_FALLBACK   no hit on either strand (the reference calls bwt_splice_match)
 *   HSA_RF_NFILTER   skipped by the #N > max_diff filter (bwtaln.c:314-317); the
 *                    reference leaves such a bwa_seq_t untouched
 *   HSA_RF_POLYAT    skipped by the first-15-bases filter (bwtaln.c:324-325)
 * splice_opt (optional, n entries): max_diff and seed_len of the option block the
 * reference hands to bwt_splice_match for each fallback read.  Hits: 9 u32 per
 * bwt_aln1_t, *hits malloc'd (hsa_free). */
#define HSA_RF_NFILTER  0x10u
#define HSA_RF_POLYAT   0x20u
long hsa_cal_sa_reg_gap_flat(hsa_index_t *ix, gap_opt_t *opt, int n, const uint32_t *lens, const uint64_t *offs,
                             const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                             uint64_t *hit_off, uint32_t **hits, int32_t *splice_opt, hsa_stats_t *stats);
/* The same over n_ix device slots (indexes of the same BWT, see hsa_gpu_set_devices). */
long hsa_cal_sa_reg_gap_multi(hsa_index_t *const *ix, int n_ix, gap_opt_t *opt, int n, const uint32_t *lens,
                              const uint64_t *offs, const uint8_t *codes, size_t codes_len, int32_t *n_aln,
                              uint32_t *flags, uint64_t *hit_off, uint32_t **hits, int32_t *splice_opt,
                              hsa_stats_t *stats);

#ifdef __cplusplus
}
#endif
#endif
