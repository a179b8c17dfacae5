/* bwtaln_gpu.h -- internals shared by the reference-ABI host sources (bwtaln_gpu.c,
 * bwtgap_gpu.c).  Not part of the public boundary (include/). */
#ifndef BWTALN_GPU_H
#define BWTALN_GPU_H
#include <stdio.h>
#include <stdlib.h>

#include "../../include/hsa_bwtaln.h"

/* the device index of a loaded Idx2BWT (slot 0), attached on first use */
hsa_index_t *hsa_gpu_index_of(const Idx2BWT *bi);
/* its indexes on every device slot in use (hsa_gpu_set_devices); *n = slot count */
hsa_index_t *const *hsa_gpu_slots_of(const Idx2BWT *bi, int *n);
/* an error message for hsa_last_error() set from C (the library's buffer is per thread) */
void hsa_gpu_set_error_text(const char *msg);
/* Direct calls into slot 0's index from the reference-ABI entry points (a splice
 * table miss, a one-off extension or SA lookup, the SAM stage's lookups) share that
 * index's staging buffers, events and stream: they hold this (recursive) lock, so that
 * the splice runner's worker threads never interleave two of them. */
void hsa_gpu_lock(void);
void hsa_gpu_unlock(void);
/* the reference's convention for unrecoverable errors: message + exit(1) */
void hsa_gpu_fatal(const char *what, long rc) __attribute__((noreturn));
/* A bump allocator for the per-batch splice tables: entries live until the table is
 * cleared, so they come from 4 MiB blocks freed together. */
typedef struct hsa_arena_blk { struct hsa_arena_blk *next; size_t used, cap; } hsa_arena_blk;
typedef struct { hsa_arena_blk *head; } hsa_arena_t;
static inline void *hsa_arena_alloc(hsa_arena_t *a, size_t n)
{
    n = (n + 15) & ~(size_t)15;
    if (!a->head || a->head->used + n > a->head->cap) {
        const size_t cap = n > ((size_t)4 << 20) ? n : ((size_t)4 << 20);
        hsa_arena_blk *b = (hsa_arena_blk *)malloc(sizeof(hsa_arena_blk) + 16 + cap);
        if (!b) { fprintf(stderr, "[hsa] out of host memory\n"); exit(1); }
        b->next = a->head; b->used = 0; b->cap = cap;
        a->head = b;
    }
    void *p = (char *)(a->head + 1) + 16 + a->head->used;
    a->head->used += n;
    return p;
}
static inline void hsa_arena_free(hsa_arena_t *a)
{
    while (a->head) { hsa_arena_blk *n = a->head->next; free(a->head); a->head = n; }
}

/* monotonic seconds (timing logs) */
double hsa_now(void);
/* aln_score (bwtgap.h) */
int hsa_aln_score(const gap_opt_t *o, int m, int g, int e);
/* the search options of one option block (the fields bwt_match_gap reads) */
hsa_regime_t hsa_regime_of(const gap_opt_t *o, int n_stacks, int max_diff);

/* splice prefetch (bwtgap_gpu.c; bwtaln_gpu.c refers to them weakly, so that a host
 * that takes only bwtaln_gpu.o still links) */
int hsa_splice_prefetch_active(void);
int hsa_splice_prefetch(const Idx2BWT *bi, int n, bwt_aux_t *const *aux);
void hsa_splice_memo_clear(void);
void hsa_splice_memo_stats(uint64_t *hits, uint64_t *misses);
void hsa_splice_table_stats(uint64_t *w_hits, uint64_t *w_misses, uint64_t *sa_hits, uint64_t *sa_misses);
/* the prefetch table's answers for the read the calling thread works on */
void hsa_splice_set_read(int r);
void hsa_splice_prefetch_warm(const Idx2BWT *bi);
void hsa_splice_warm(int n_coroutines);
int hsa_splice_table_width(const Idx2BWT *bi, int len, const ubyte_t *str, bwt_width_t *width, int type, int *ret);
int hsa_splice_table_sa(const Idx2BWT *bi, uint32_t idx, uint32_t o[3]);

/* the splice path's seed extensions and its batched runner (bwtext_gpu.c; referred to
 * weakly as well) */
typedef struct {
    const ubyte_t *seq;        /* the read (bwa_seq_t.seq) */
    int len;
    gap_opt_t opt;             /* local_opt as bwt_splice_match receives it for this read */
} hsa_splice_read_t;
int hsa_splice_extend_active(void);
void hsa_splice_sa_clear(void);
void hsa_splice_sa_stats(uint64_t *hits, uint64_t *misses);
void hsa_splice_sa_position(Idx2BWT *bi, unsigned int sa_index, unsigned int *seq_id, unsigned int *ori_pos,
                            unsigned int *occ_pos);
int hsa_splice_width_active(void);
long hsa_splice_run(const Idx2BWT *bi, struct bwt_array_t *arr, int max_len, int n_stacks, int n,
                    const hsa_splice_read_t *reads, bwt_aln1_t **out, int *n_out);

#endif
