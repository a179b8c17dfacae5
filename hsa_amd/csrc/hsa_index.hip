// hsa_index.hip -- device index (rank blocks) and the rank/step/width primitives.
//
// The reference keeps, per BWT direction, a 2-bit code array plus two sampled
// Occ tables (occValue every 256 chars as 16-bit pairs, occValueMajor every 65 536;
// BWT.c:1018-1059) and answers a rank with two dependent-ish loads and an SSE
// popcount (BWT.c:532-679).  Here one 16-byte block carries the absolute counts
// and the 16 codes they precede (hsa_device.h), so one rank query = one load.
#include <chrono>
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"
#include "hsa_trie.h"

static thread_local char g_err[1024] = "";
int g_waves_per_cu = 16;
int g_pool_entries = 0;      // 0: 8192 per lane, 32768 when gap opens are allowed
// k_search: when a wave runs the strand-end / next-read paths of its waiting lanes:
// at most HSA_BATCH_K waiting lanes, or HSA_BATCH_IDLE lane-iterations of waiting
// (overrides for A/B runs)
int g_batch_k = getenv("HSA_BATCH_K") ? atoi(getenv("HSA_BATCH_K")) : 32;
int g_batch_idle = getenv("HSA_BATCH_IDLE") ? atoi(getenv("HSA_BATCH_IDLE")) : 768;
int g_hit_cap = 64;

void hsa_set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

extern "C" const char *hsa_last_error(void) { return g_err; }
extern "C" void hsa_gpu_set_error_text(const char *msg) { hsa_set_error("%s", msg); }

extern "C" int hsa_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" void hsa_free(void *p) { free(p); }

extern "C" int hsa_configure(int waves_per_cu, int pool_entries, int hit_cap)
{
    if (waves_per_cu > 0) g_waves_per_cu = waves_per_cu;
    if (pool_entries > 0) {
        if (pool_entries > 65535) { hsa_set_error("pool_entries > 65535"); return HSA_E_ARG; }
        g_pool_entries = pool_entries;
    } else if (pool_entries < 0) {
        g_pool_entries = 0;              // back to the per-regime default
    }
    if (hit_cap > 0) g_hit_cap = hit_cap;
    return 0;
}

// HSA_VERBOSE: device allocations that take more than 5 ms (a first batch's stall)
static void hsa_log_alloc(const char *what, size_t bytes, std::chrono::steady_clock::time_point t0)
{
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > 5.0 && getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] %s: hipMalloc of %.2f GB took %.1f ms\n", what, bytes / 1e9, ms);
}

// A new device buffer of `bytes` in *out, and the old one (*old, contents not kept)
// freed: allocated BEFORE the old one is freed where HBM allows, since a large hipMalloc
// right after the hipFree of a large block was measured at ~115 ms per GB (6.9 s for a
// first batch's 59.6 GB search scratch), a fresh one at a few ms.  *old is null after.
int hsa_realloc_device(void **out, void **old, size_t bytes)
{
    *out = nullptr;
    if (hipMalloc(out, bytes) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        (void)hipFree(*old);                       // no room for both: the slow path
        *old = nullptr;
        if (hipMalloc(out, bytes) != hipSuccess) {
            (void)hipGetLastError();
            *out = nullptr;
            hsa_set_error("hipMalloc(%zu) failed", bytes);
            return HSA_E_MEM;
        }
        return 0;
    }
    (void)hipFree(*old);
    *old = nullptr;
    return 0;
}

int hsa_grow(void **p, size_t *cap, size_t need)
{
    if (need <= *cap && *p) return 0;
    size_t n = need + need / 4 + 4096;
    const auto t0 = std::chrono::steady_clock::now();
    void *np = nullptr;
    *cap = 0;
    if (hsa_realloc_device(&np, p, n)) return HSA_E_MEM;
    *p = np;
    *cap = n;
    hsa_log_alloc("buffer", n, t0);
    return 0;
}

void hsa_scratch_free(SearchScratch &s)
{
    (void)hipFree(s.pool); (void)hipFree(s.nxt); (void)hipFree(s.hbuf);
    const size_t lb = s.link_bytes;
    s = SearchScratch();
    s.link_bytes = lb;
}

extern "C" int hsa_index_release_scratch(hsa_index_t *ix)
{
    if (!ix) { hsa_set_error("hsa_index_release_scratch: null handle"); return HSA_E_ARG; }
    (void)hipSetDevice(ix->device);
    HSA_HIP(hipStreamSynchronize(ix->stream));
    hsa_scratch_free(ix->main); hsa_scratch_free(ix->big); hsa_scratch_free(ix->huge);
    void **bufs[] = {&ix->d_pf, &ix->d_pf2, &ix->d_sp, &ix->d_any, &ix->d_any_aux, &ix->d_help};
    size_t *caps[] = {&ix->d_pf_cap, &ix->d_pf2_cap, &ix->d_sp_cap, &ix->d_any_cap, &ix->d_any_aux_cap, &ix->d_help_cap};
    for (int i = 0; i < 6; ++i) {
        if (*bufs[i]) (void)hipFree(*bufs[i]);
        *bufs[i] = nullptr;
        *caps[i] = 0;
    }
    return 0;
}

int hsa_scratch_reserve(SearchScratch &s, size_t lanes, size_t pcap, size_t hcap, size_t link_bytes)
{
    const size_t pe = lanes * pcap, he = lanes * hcap;
    // The pool (+ links) and the staged hits grow separately: a wide pass that needs more
    // hit slots must not free and re-allocate a deep pass's tens of GB of pool (measured:
    // 6.9 s for a 59.6 GB hipMalloc right after the hipFree of the old one)
    auto fail = [&]() {
        hsa_set_error("scratch allocation failed (lanes %zu, pool %zu, hits %zu)", lanes, pcap, hcap);
        (void)hipGetLastError();    // not sticky: a caller may free memory and go on
        hsa_scratch_free(s);
        return HSA_E_MEM;
    };
    if (!s.pool || pe > s.pool_entries || link_bytes != s.link_bytes) {
        const size_t npe = pe > s.pool_entries ? pe : s.pool_entries;
        const auto t0 = std::chrono::steady_clock::now();
        void *np = nullptr, *nn = nullptr;
        if (hsa_realloc_device(&np, (void **)&s.pool, npe * sizeof(uint4)) ||
            hsa_realloc_device(&nn, &s.nxt, npe * link_bytes)) {
            (void)hipFree(np);
            return fail();
        }
        s.pool = (uint4 *)np; s.nxt = nn;
        s.pool_entries = npe;
        s.link_bytes = link_bytes;
        hsa_log_alloc("search scratch pool", npe * (sizeof(uint4) + link_bytes), t0);
    }
    if (!s.hbuf || he > s.hit_entries) {
        const size_t nhe = he > s.hit_entries ? he : s.hit_entries;
        const auto t0 = std::chrono::steady_clock::now();
        void *nh = nullptr;
        if (hsa_realloc_device(&nh, (void **)&s.hbuf, nhe * 9 * sizeof(uint32_t))) return fail();
        s.hbuf = (uint32_t *)nh;
        s.hit_entries = nhe;
        hsa_log_alloc("search scratch hits", nhe * 9 * sizeof(uint32_t), t0);
    }
    return 0;
}

// ---------------------------------------------------------------- layout build
__global__ void k_msb_to_lsb(uint32_t *w, size_t n, uint32_t T)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = w[i];
    x = (x >> 16) | (x << 16);
    x = ((x & 0xFF00FF00u) >> 8) | ((x & 0x00FF00FFu) << 8);
    x = ((x & 0xF0F0F0F0u) >> 4) | ((x & 0x0F0F0F0Fu) << 4);
    x = ((x & 0xCCCCCCCCu) >> 2) | ((x & 0x33333333u) << 2);
    if (i == n - 1 && (T & 15)) x &= (1u << (2 * (T & 15))) - 1u;   // BWTClearTrailingBwtCode
    w[i] = x;
}

struct U4 { uint32_t a, b, c, d; };
struct U4Plus {
    __host__ __device__ U4 operator()(const U4 &x, const U4 &y) const
    {
        return U4{x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d};
    }
};

// Counts of A, C, G among the valid characters of code word b (the last word may be
// partial: its padding codes are 0 but are not characters, so A = valid - C - G - T).
struct WordCounts {
    const uint32_t *code;
    size_t nwords;
    uint64_t T;
    __host__ __device__ U4 operator()(size_t b) const
    {
        const uint32_t v = b < nwords ? code[b] : 0u;
        const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
        const uint32_t t3 = __popc(lo & hi), t1 = __popc(lo) - t3, t2 = __popc(hi) - t3;
        const uint64_t s = (uint64_t)b * HSA_BLK_CHARS;
        const uint32_t valid = s >= T ? 0u : (uint32_t)((T - s) < HSA_BLK_CHARS ? (T - s) : HSA_BLK_CHARS);
        return U4{valid - t1 - t2 - t3, t1, t2, 0u};
    }
};

// block b = (Occ A, C, G over [0, 16b) from the scan, code word b).  The scan's u32
// sums wrap past 2^32 characters: the counts are then kept modulo 2^32 and the wrap
// table (build_wraps) supplies the high part.
__global__ void k_block_codes(const uint32_t *__restrict__ code, size_t nwords, size_t nblk, uint4 *__restrict__ blk)
{
    const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    blk[b].w = b < nwords ? code[b] : 0u;
}

static int build_blocks(hsa_index *ix, int dir, uint64_t T, const uint32_t *d_code_lsb, hipStream_t st)
{
    const size_t nwords = ((size_t)T + 15) / 16;
    const size_t nblk = (size_t)T / HSA_BLK_CHARS + 2;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    HSA_HIP(hipMalloc(&ix->blk_base[dir], nblk * 16 + HSA_WRAP_HEAD));
    HSA_HIP(hipMemset(ix->blk_base[dir], 0, HSA_WRAP_HEAD));       // no wraps
    ix->blk[dir] = reinterpret_cast<uint4 *>(static_cast<char *>(ix->blk_base[dir]) + HSA_WRAP_HEAD);
    ix->nblk[dir] = nblk;
    auto in = rocprim::make_transform_iterator(rocprim::make_counting_iterator<size_t>(0),
                                               WordCounts{d_code_lsb, nwords, T});
    U4 *out = reinterpret_cast<U4 *>(ix->blk[dir]);
    const U4 zero{0, 0, 0, 0};
    HSA_HIP(rocprim::exclusive_scan(tmp, tmp_bytes, in, out, zero, nblk, U4Plus(), st));
    HSA_HIP(hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 16));
    HSA_HIP(rocprim::exclusive_scan(tmp, tmp_bytes, in, out, zero, nblk, U4Plus(), st));
    k_block_codes<<<(unsigned)((nblk + 255) / 256), 256, 0, st>>>(d_code_lsb, nwords, nblk, ix->blk[dir]);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipStreamSynchronize(st));
    (void)hipFree(tmp);
    return 0;
}

// The wrap table of RankDir64: block b > 0 is a wrap of base c when its low count word
// is below block b - 1's (counts grow by <= 16 per block).  At most HSA_MAX_WRAPS per
// base under HSA_WIDE_MAX_T characters; the slots fill in any order and are sorted on
// the host.
__global__ void k_find_wraps(const uint4 *__restrict__ blk, size_t nblk, unsigned *cnt, unsigned *out)
{
    const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0 || b >= nblk) return;
    const uint4 x = blk[b - 1], y = blk[b];
    const uint32_t lo[3][2] = {{x.x, y.x}, {x.y, y.y}, {x.z, y.z}};
    for (int c = 0; c < 3; ++c)
        if (lo[c][1] < lo[c][0]) {
            const unsigned k = atomicAdd(&cnt[c], 1u);
            if (k < HSA_MAX_WRAPS) out[c * HSA_MAX_WRAPS + k] = (unsigned)b;
        }
}

static int build_wraps(hsa_index *ix, int dir, hipStream_t st)
{
    unsigned *d = nullptr;
    const size_t words = 3 + 3 * HSA_MAX_WRAPS;
    HSA_HIP(hipMalloc(&d, words * 4));
    HSA_HIP(hipMemsetAsync(d, 0, words * 4, st));
    const size_t nblk = ix->nblk[dir];
    k_find_wraps<<<(unsigned)((nblk + 255) / 256), 256, 0, st>>>(ix->blk[dir], nblk, d, d + 3);
    unsigned h[3 + 3 * HSA_MAX_WRAPS];
    const hipError_t e1 = hipGetLastError();
    const hipError_t e2 = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, st);
    const hipError_t e3 = hipStreamSynchronize(st);
    (void)hipFree(d);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) { hsa_set_error("wrap table"); return HSA_E_HIP; }
    uint32_t tab[HSA_WRAP_HEAD / 4] = {};
    uint32_t n = 0;
    for (uint32_t c = 0; c < 3; ++c) {
        if (h[c] > HSA_MAX_WRAPS) { hsa_set_error("more than %u count wraps", HSA_MAX_WRAPS); return HSA_E_ARG; }
        for (uint32_t k = 0; k < h[c]; ++k, ++n) {
            tab[2 + 2 * n] = h[3 + c * HSA_MAX_WRAPS + k];
            tab[3 + 2 * n] = c;
        }
    }
    for (uint32_t i = 1; i < n; ++i)                 // insertion sort by block, <= 45 entries
        for (uint32_t j = i; j > 0 && tab[2 + 2 * j] < tab[2 * j]; --j) {
            uint32_t *x = tab + 2 + 2 * j, *y = tab + 2 * j;
            const uint32_t t0 = x[0], t1 = x[1];
            x[0] = y[0]; x[1] = y[1]; y[0] = t0; y[1] = t1;
        }
    tab[0] = n;
    ix->any_wrap[dir] = n > 0;
    HSA_HIP(hipMemcpy((void *)hsa_wrap_table(ix->blk[dir]), tab, sizeof tab, hipMemcpyHostToDevice));
    return 0;
}

RankDir64 hsa_rank_dir64(const hsa_index *ix, int dir)
{
    return RankDir64{ix->blk[dir], dir ? ix->risa0_64 : ix->isa0_64, ix->any_wrap[dir] ? 1u : 0u};
}

// The root width trie of hsa_trie.h, level by level on the index's stream: HSA_TRIE_DEPTH
// levels (0 = none; by default 12, less for a text shorter than 4^(D-1) characters, whose
// deeper levels would hold mostly empty strings).
template <typename IT, typename RD>
static int build_tries_t(hsa_index *ix, RD rev, IT T, const IT *C)
{
    uint32_t D = HSA_TRIE_DEFAULT_DEPTH;
    if (const char *e = getenv("HSA_TRIE_DEPTH")) {        // as asked (tests: tries deeper than the text)
        D = (uint32_t)atoi(e);
        if (D > HSA_TRIE_MAX_DEPTH) D = HSA_TRIE_MAX_DEPTH;
    } else {
        while (D > 0 && (1ull << (2 * D)) > 4ull * (uint64_t)T) --D;
    }
    ix->trie_depth = 0;
    if (D == 0) return 0;
    const size_t ws = sizeof(IT) == 4 ? 8 : 16;
    const size_t nw = trie_base(D + 1);
    // the trie only saves rank steps: without the memory for it the index still serves
    // every search (rank steps only), so an allocation failure is not an error here
    if (hipMalloc(&ix->d_trie_w, nw * ws) != hipSuccess) {
        (void)hipGetLastError();
        ix->d_trie_w = nullptr;
        if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] root trie: no device memory for it, rank steps only\n");
        return 0;
    }
    TrieC<IT> Cv;
    for (int c = 0; c < 4; ++c) Cv.v[c] = C[c];
    unsigned *d_bad = nullptr, bad = 0;
    HSA_HIP(hipMalloc(&d_bad, 4));
    HSA_HIP(hipMemsetAsync(d_bad, 0, 4, ix->stream));
    for (uint32_t d = 0; d < D; ++d) {
        const unsigned nb = (unsigned)(((1ull << (2 * d)) + 255) / 256);
        hipLaunchKernelGGL((k_trie_width_level<IT, RD>), dim3(nb), dim3(256), 0, ix->stream, rev, T, Cv, d, ix->d_trie_w,
                           d_bad);
        HSA_HIP(hipGetLastError());
    }
    HSA_HIP(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    (void)hipFree(d_bad);
    if (bad) {                      // the two BWTs disagree: no trie (rank steps only)
        if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] root trie: intervals past the text, not kept\n");
        (void)hipFree(ix->d_trie_w);
        ix->d_trie_w = nullptr;
        return 0;
    }
    ix->trie_depth = D;
    ix->trie_wide = sizeof(IT) == 8;
    ix->trie_bytes = nw * ws;
    return 0;
}

static int build_tries(hsa_index *ix)
{
    if (ix->wide) return build_tries_t<uint64_t, RankDir64>(ix, hsa_rank_dir64(ix, 1), ix->T64, ix->C64);
    return build_tries_t<uint32_t, RankDir>(ix, RankDir{ix->blk[1], ix->risa0}, ix->T, ix->C);
}

int hsa_need32(const hsa_index *ix)
{
    if (!ix->is64) return 0;
    hsa_set_error("the index text has 2^32 characters or more: use the 64-bit entry points (*64)");
    return HSA_E_ARG;
}

static int index_init(int device, hsa_index **out)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        hsa_set_error("no HIP device visible");
        return HSA_E_NODEV;
    }
    if (device < 0 || device >= n) { hsa_set_error("device %d out of range (%d)", device, n); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(device));
    hsa_index *ix = new hsa_index();
    ix->device = device;
    hipDeviceProp_t prop;
    HSA_HIP(hipGetDeviceProperties(&prop, device));
    ix->n_cu = prop.multiProcessorCount;
    HSA_HIP(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking));
    HSA_HIP(hipEventCreate(&ix->ev0));
    HSA_HIP(hipEventCreate(&ix->ev1));
    HSA_HIP(hipEventCreate(&ix->evm));
    HSA_HIP(hipEventCreate(&ix->ev_sp));
    ix->ev_split = ix->evm;
    HSA_HIP(hipMalloc(&ix->d_ctr, 16 * sizeof(uint64_t)));
    *out = ix;
    return 0;
}

extern "C" int hsa_index_create_device(int device, uint32_t T, uint32_t isa0, const uint32_t C[5],
                                       const uint32_t *d_code_lsb, uint32_t rT, uint32_t risa0,
                                       const uint32_t rC[5], const uint32_t *d_rcode_lsb, hsa_index_t **out)
{
    hsa_index *ix = nullptr;
    int rc = index_init(device, &ix);
    if (rc) return rc;
    ix->T = T; ix->isa0 = isa0; memcpy(ix->C, C, sizeof ix->C);
    ix->rT = rT; ix->risa0 = risa0; memcpy(ix->rC, rC, sizeof ix->rC);
    if ((rc = build_blocks(ix, 0, T, d_code_lsb, ix->stream)) ||
        (rc = build_blocks(ix, 1, rT, d_rcode_lsb, ix->stream)) || (rc = build_tries(ix))) {
        hsa_index_free(ix);
        return rc;
    }
    *out = ix;
    return 0;
}

extern "C" int hsa_index_create_device64(int device, uint64_t T, uint64_t isa0, const uint64_t C[5],
                                         const uint32_t *d_code_lsb, uint64_t rT, uint64_t risa0, const uint64_t rC[5],
                                         const uint32_t *d_rcode_lsb, hsa_index_t **out)
{
    if (!C || !rC || !d_code_lsb || !d_rcode_lsb || !out) { hsa_set_error("null argument"); return HSA_E_ARG; }
    if (T == 0 || rT == 0 || C[4] != T || rC[4] != rT || isa0 > T || risa0 > rT) {
        hsa_set_error("inconsistent lengths (C[4] must equal T, isa0 <= T)");
        return HSA_E_ARG;
    }
    if (T >= HSA_WIDE_MAX_T || rT >= HSA_WIDE_MAX_T) { hsa_set_error("text of 2^36 characters or more"); return HSA_E_ARG; }
    hsa_index *ix = nullptr;
    int rc = index_init(device, &ix);
    if (rc) return rc;
    ix->wide = true;
    ix->is64 = T > 0xFFFFFFFFull - 1 || rT > 0xFFFFFFFFull - 1;
    ix->T64 = T; ix->isa0_64 = isa0; memcpy(ix->C64, C, sizeof ix->C64);
    ix->rT64 = rT; ix->risa0_64 = risa0; memcpy(ix->rC64, rC, sizeof ix->rC64);
    if (!ix->is64) {       // the 32-bit entry points serve the same index
        ix->T = (uint32_t)T; ix->isa0 = (uint32_t)isa0; ix->rT = (uint32_t)rT; ix->risa0 = (uint32_t)risa0;
        for (int c = 0; c < 5; ++c) { ix->C[c] = (uint32_t)C[c]; ix->rC[c] = (uint32_t)rC[c]; }
    }
    if ((rc = build_blocks(ix, 0, T, d_code_lsb, ix->stream)) || (rc = build_blocks(ix, 1, rT, d_rcode_lsb, ix->stream)) ||
        (rc = build_wraps(ix, 0, ix->stream)) || (rc = build_wraps(ix, 1, ix->stream)) || (rc = build_tries(ix))) {
        hsa_index_free(ix);
        return rc;
    }
    *out = ix;
    return 0;
}

extern "C" int hsa_index_create(int device, uint32_t T, uint32_t isa0, const uint32_t C[5], const uint32_t *code,
                                uint32_t rT, uint32_t risa0, const uint32_t rC[5], const uint32_t *rcode,
                                hsa_index_t **out)
{
    if (!code || !rcode || !C || !rC || !out) { hsa_set_error("null argument"); return HSA_E_ARG; }
    if (C[4] != T || rC[4] != rT) { hsa_set_error("C[4] must equal the text length"); return HSA_E_ARG; }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) { hsa_set_error("no HIP device visible"); return HSA_E_NODEV; }
    HSA_HIP(hipSetDevice(device));
    size_t nw = ((size_t)T + 15) / 16, rnw = ((size_t)rT + 15) / 16;
    uint32_t *d = nullptr, *rd = nullptr;
    HSA_HIP(hipMalloc(&d, nw * 4 + 64));
    HSA_HIP(hipMalloc(&rd, rnw * 4 + 64));
    HSA_HIP(hipMemcpy(d, code, nw * 4, hipMemcpyHostToDevice));
    HSA_HIP(hipMemcpy(rd, rcode, rnw * 4, hipMemcpyHostToDevice));
    k_msb_to_lsb<<<(unsigned)((nw + 255) / 256), 256>>>(d, nw, T);
    k_msb_to_lsb<<<(unsigned)((rnw + 255) / 256), 256>>>(rd, rnw, rT);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipDeviceSynchronize());
    int rc = hsa_index_create_device(device, T, isa0, C, d, rT, risa0, rC, rd, out);
    (void)hipFree(d); (void)hipFree(rd);
    return rc;
}

// A second handle on the same resident index for concurrent passes: the read-only
// arrays are shared, the stream, events, scratch and staging are the clone's own.
extern "C" int hsa_index_clone(hsa_index_t *src, hsa_index_t **out)
{
    if (!src || !out) { hsa_set_error("null argument"); return HSA_E_ARG; }
    hsa_index *root = src->parent ? src->parent : src;
    hsa_index *ix = nullptr;
    int rc = index_init(root->device, &ix);
    if (rc) return rc;
    ix->T = root->T; ix->isa0 = root->isa0; memcpy(ix->C, root->C, sizeof ix->C);
    ix->rT = root->rT; ix->risa0 = root->risa0; memcpy(ix->rC, root->rC, sizeof ix->rC);
    for (int d = 0; d < 2; ++d) {
        ix->blk[d] = root->blk[d]; ix->blk_base[d] = root->blk_base[d]; ix->nblk[d] = root->nblk[d];
        ix->any_wrap[d] = root->any_wrap[d];
    }
    ix->wide = root->wide; ix->is64 = root->is64;
    ix->T64 = root->T64; ix->isa0_64 = root->isa0_64; memcpy(ix->C64, root->C64, sizeof ix->C64);
    ix->rT64 = root->rT64; ix->risa0_64 = root->risa0_64; memcpy(ix->rC64, root->rC64, sizeof ix->rC64);
    ix->d_sa = root->d_sa; ix->d_blocks = root->d_blocks;
    ix->d_text = root->d_text; ix->text_words = root->text_words; ix->dna_len = root->dna_len;
    ix->sa_interval = root->sa_interval; ix->n_blocks = root->n_blocks;
    ix->d_trie_w = root->d_trie_w;
    ix->trie_depth = root->trie_depth;
    ix->trie_wide = root->trie_wide; ix->trie_bytes = root->trie_bytes;
    ix->parent = root;
    __atomic_add_fetch(&root->n_clones, 1, __ATOMIC_ACQ_REL);
    *out = ix;
    return 0;
}

int hsa_need_unshared(const hsa_index *ix, const char *what)
{
    if (!ix->parent && !ix->n_clones) return 0;
    hsa_set_error("%s: %s", what, ix->parent ? "not on a clone (call it on the index before cloning)"
                                              : "the index has live clones (free them first)");
    return HSA_E_ARG;
}

extern "C" void hsa_index_free(hsa_index_t *ix)
{
    if (!ix) return;
    if (!ix->parent) {
        // live clones still read the shared arrays: the free is deferred to the last
        // clone's (the handle stays valid for them, not for the caller).  Clones may be
        // freed from other threads: the flag is published before the count is re-read,
        // and the clone that takes the count to 0 reads the flag after its decrement.
        __atomic_store_n(&ix->free_pending, true, __ATOMIC_SEQ_CST);
        if (__atomic_load_n(&ix->n_clones, __ATOMIC_SEQ_CST) > 0) return;
        // no clone left (or none ever): free now, unless the last clone's free races us
        // to it (exactly one of the two sees free_pending still set and takes it)
        if (!__atomic_exchange_n(&ix->free_pending, false, __ATOMIC_SEQ_CST)) return;
    }
    (void)hipSetDevice(ix->device);
    hsa_index *orphan = nullptr;
    if (ix->parent) {           // the shared arrays stay with the parent
        if (__atomic_sub_fetch(&ix->parent->n_clones, 1, __ATOMIC_SEQ_CST) == 0 &&
            __atomic_exchange_n(&ix->parent->free_pending, false, __ATOMIC_SEQ_CST))
            orphan = ix->parent;
        ix->blk_base[0] = ix->blk_base[1] = nullptr;
        ix->d_sa = ix->d_blocks = nullptr;
        ix->d_text = nullptr;
        ix->d_trie_w = nullptr;
    }
    (void)hipFree(ix->blk_base[0]); (void)hipFree(ix->blk_base[1]);
    hsa_scratch_free(ix->main); hsa_scratch_free(ix->big); hsa_scratch_free(ix->huge);
    if (ix->d_ovf2) (void)hipFree(ix->d_ovf2);
    if (ix->d_any) (void)hipFree(ix->d_any);
    if (ix->d_any_aux) (void)hipFree(ix->d_any_aux);
    if (ix->d_split) (void)hipFree(ix->d_split);
    if (ix->d_help) (void)hipFree(ix->d_help);
    if (ix->d_fwd) (void)hipFree(ix->d_fwd);
    if (ix->d_pf) (void)hipFree(ix->d_pf);
    if (ix->d_pf2) (void)hipFree(ix->d_pf2);
    if (ix->h_pf) (void)hipHostFree(ix->h_pf);
    (void)hipFree(ix->d_in); (void)hipFree(ix->d_out); (void)hipFree(ix->d_ctr); (void)hipFree(ix->d_wrows); (void)hipFree(ix->d_ovf); (void)hipFree(ix->d_seed); (void)hipFree(ix->d_ext); (void)hipFree(ix->d_slices);
    (void)hipFree(ix->d_sa); (void)hipFree(ix->d_blocks); (void)hipFree(ix->d_text);
    if (ix->d_sp) (void)hipFree(ix->d_sp);
    (void)hipFree(ix->d_trie_w);
    if (ix->ev0) (void)hipEventDestroy(ix->ev0);
    if (ix->ev1) (void)hipEventDestroy(ix->ev1);
    if (ix->evm) (void)hipEventDestroy(ix->evm);
    if (ix->ev_sp) (void)hipEventDestroy(ix->ev_sp);
    for (int i = 0; i < hsa_index::PASS_RING; ++i)
        for (int j = 0; j < 3; ++j)
            if (ix->pev[i][j]) (void)hipEventDestroy(ix->pev[i][j]);
    if (ix->stream) (void)hipStreamDestroy(ix->stream);
    delete ix;
    if (orphan) hsa_index_free(orphan);     // a parent freed before its last clone
}

extern "C" size_t hsa_index_bytes(const hsa_index_t *ix)
{
    return (ix->nblk[0] + ix->nblk[1]) * 16;
}
extern "C" int hsa_index_is64(const hsa_index_t *ix) { return ix->is64 ? 1 : 0; }
extern "C" int hsa_index_trie(const hsa_index_t *ix, uint32_t *depth, uint32_t *sdepth, size_t *bytes)
{
    if (depth) *depth = ix->trie_depth;
    if (sdepth) *sdepth = 0;                   // no search trie (hsa_trie.h)
    if (bytes) *bytes = ix->trie_bytes;
    return 0;
}
extern "C" int hsa_index_device(const hsa_index_t *ix) { return ix->device; }
extern "C" void *hsa_index_stream(const hsa_index_t *ix) { return (void *)ix->stream; }

// ---------------------------------------------------------------- primitives
__global__ void k_occ4(RankDir d, const uint32_t *pos, size_t n, uint32_t *out)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t o[4];
    hsa_occ4(d, pos[i], o);
    out[4 * i] = o[0]; out[4 * i + 1] = o[1]; out[4 * i + 2] = o[2]; out[4 * i + 3] = o[3];
}

__global__ void k_occ4_64(RankDir64 d, const uint64_t *pos, size_t n, uint64_t *out)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t a[4], b[4];
    occ_pair(d, pos[i], pos[i], a, b);
    out[4 * i] = a[0]; out[4 * i + 1] = a[1]; out[4 * i + 2] = a[2]; out[4 * i + 3] = a[3];
}

extern "C" int hsa_occ4_batch64(hsa_index_t *ix, int dir, size_t n, const uint64_t *pos, uint64_t *occ)
{
    if (dir < 0 || dir > 1) { hsa_set_error("dir"); return HSA_E_ARG; }
    if (!ix->wide) { hsa_set_error("not a 64-bit index (hsa_index_create_device64)"); return HSA_E_ARG; }
    const uint64_t T = dir ? ix->rT64 : ix->T64;
    for (size_t i = 0; i < n; ++i)
        if (pos[i] > T + 1) { hsa_set_error("position %llu > T + 1", (unsigned long long)pos[i]); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, n * 8 + 16)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, n * 32 + 16)))
        return rc;
    HSA_HIP(hipMemcpyAsync(ix->d_in, pos, n * 8, hipMemcpyHostToDevice, ix->stream));
    const RankDir64 d = hsa_rank_dir64(ix, dir);
    if (n) k_occ4_64<<<(unsigned)((n + 255) / 256), 256, 0, ix->stream>>>(d, (const uint64_t *)ix->d_in, n, (uint64_t *)ix->d_out);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipMemcpyAsync(occ, ix->d_out, n * 32, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    return 0;
}

extern "C" int hsa_occ4_batch(hsa_index_t *ix, int dir, size_t n, const uint32_t *pos, uint32_t *occ)
{
    if (dir < 0 || dir > 1) { hsa_set_error("dir"); return HSA_E_ARG; }
    if (int rc0 = hsa_need32(ix)) return rc0;
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;                      // d_in is reused below
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, n * 4 + 16)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, n * 16 + 16)))
        return rc;
    HSA_HIP(hipMemcpyAsync(ix->d_in, pos, n * 4, hipMemcpyHostToDevice, ix->stream));
    RankDir d{ix->blk[dir], dir ? ix->risa0 : ix->isa0};
    if (n) k_occ4<<<(unsigned)((n + 255) / 256), 256, 0, ix->stream>>>(d, (const uint32_t *)ix->d_in, n, (uint32_t *)ix->d_out);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipMemcpyAsync(occ, ix->d_out, n * 16, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    return 0;
}

// BWTAllSARangesBackward_Bidirection (2BWT-Interface.c:235-272)
__global__ void k_step(RankDir d, const uint32_t *C, const uint32_t *in, size_t n, uint32_t *out)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = in[4 * i], l = in[4 * i + 1], rl = in[4 * i + 3];
    uint32_t a[4], b[4];
    hsa_occ_pair(d, k, l + 1, a, b);
    uint32_t oc[4];
    oc[3] = 0;
    for (int c = 2; c >= 0; --c) oc[c] = oc[c + 1] + b[c + 1] - a[c + 1];
    uint32_t *o = out + 16 * i;
    for (int c = 0; c < 4; ++c) {
        uint32_t nk = C[c] + a[c] + 1, nl = C[c] + b[c];
        uint32_t nrl = rl - oc[c];
        o[c] = nk; o[4 + c] = nl; o[12 + c] = nrl; o[8 + c] = nrl - (nl - nk);
    }
}

extern "C" int hsa_step_batch(hsa_index_t *ix, size_t n, const uint32_t *klrr, uint32_t *out16)
{
    if (int rc0 = hsa_need32(ix)) return rc0;
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;                      // d_in is reused below
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, n * 16 + 64)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, n * 64 + 16)))
        return rc;
    HSA_HIP(hipMemcpyAsync(ix->d_in, klrr, n * 16, hipMemcpyHostToDevice, ix->stream));
    uint32_t *dC = (uint32_t *)((char *)ix->d_in + ((n * 16 + 15) / 16) * 16);
    HSA_HIP(hipMemcpyAsync(dC, ix->C, 5 * 4, hipMemcpyHostToDevice, ix->stream));
    RankDir d{ix->blk[0], ix->isa0};
    if (n) k_step<<<(unsigned)((n + 255) / 256), 256, 0, ix->stream>>>(d, dC, (const uint32_t *)ix->d_in, n, (uint32_t *)ix->d_out);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipMemcpyAsync(out16, ix->d_out, n * 64, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    return 0;
}

// bwt_cal_width type 1 (bwtaln.c:73-98), one read per thread (test primitive;
// the search kernel has its own interleaved version).
__global__ void k_width(RankDir rev, uint32_t T, const uint32_t *C, const uint64_t *offs, const uint32_t *lens,
                        const uint64_t *woff, const uint8_t *codes, size_t n, uint32_t *w)
{
    size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t *s = codes + offs[r];
    uint32_t len = lens[r], k = 0, l = T;
    int bid = 0;
    uint32_t *o = w + woff[r];
    for (uint32_t i = 0; i < len; ++i) {
        uint8_t c = s[i];
        if (c < 4) {
            uint32_t a[4], b[4];
            hsa_occ_pair(rev, k, l + 1, a, b);
            k = C[c] + a[c] + 1;
            l = C[c] + b[c];
        }
        if (k > l || c > 3) { k = 0; l = T; ++bid; }
        o[2 * i] = l - k + 1;
        o[2 * i + 1] = (uint32_t)bid;
    }
    o[2 * len] = 0;
    o[2 * len + 1] = (uint32_t)(bid + 1);
}

// bwt_cal_width type 0 (bwtaln.c:98-115): backward on the forward BWT
// (BWTSARangeBackward, 2BWT-Interface.c:107-118) from the read's end; entries
// [1, len) and [len] = {0, ++bid} are written, entry 0 never is (the reference's loop
// stops at i > 0): it is left 0 here, and callers copy entries 1..len only.
__global__ void k_width0(RankDir fwd, uint32_t T, const uint32_t *C, const uint64_t *offs, const uint32_t *lens,
                         const uint64_t *woff, const uint8_t *codes, size_t n, uint32_t *w)
{
    size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t *s = codes + offs[r];
    const uint32_t len = lens[r];
    uint32_t k = 0, l = T;
    int bid = 0;
    uint32_t *o = w + woff[r];
    o[0] = 0; o[1] = 0;
    for (uint32_t i = len - 1; i > 0 && len > 0; --i) {
        const uint8_t c = s[i];
        if (c < 4) {
            uint32_t a, b;
            hsa_occ1_pair(fwd, k, l + 1, c, a, b);
            k = C[c] + a + 1;
            l = C[c] + b;
        }
        if (k > l || c > 3) { k = 0; l = T; ++bid; }
        o[2 * i] = l - k + 1;
        o[2 * i + 1] = (uint32_t)bid;
    }
    o[2 * len] = 0;
    o[2 * len + 1] = (uint32_t)(bid + 1);
}

static int width_batch(hsa_index_t *ix, int type, size_t n, const uint64_t *offs, const uint32_t *lens,
                       const uint8_t *codes, size_t codes_len, uint32_t *width_out)
{
    if (int rc0 = hsa_need32(ix)) return rc0;
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;                      // d_in is reused below
    uint64_t *woff = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    uint64_t tot = 0;
    for (size_t i = 0; i < n; ++i) { woff[i] = tot; tot += 2 * ((uint64_t)lens[i] + 1); }
    size_t inb = n * 8 + n * 4 + n * 8 + codes_len + 5 * 4 + 256;
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, inb)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, tot * 4 + 16))) {
        free(woff);
        return rc;
    }
    char *p = (char *)ix->d_in;
    uint64_t *d_offs = (uint64_t *)p; p += n * 8;
    uint64_t *d_woff = (uint64_t *)p; p += n * 8;
    uint32_t *d_lens = (uint32_t *)p; p += n * 4;
    uint32_t *d_C = (uint32_t *)p; p += 32;
    uint8_t *d_codes = (uint8_t *)p;
    HSA_HIP(hipMemcpyAsync(d_offs, offs, n * 8, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(d_woff, woff, n * 8, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(d_lens, lens, n * 4, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(d_C, ix->C, 20, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(d_codes, codes, codes_len, hipMemcpyHostToDevice, ix->stream));
    RankDir rev{ix->blk[1], ix->risa0}, fwd{ix->blk[0], ix->isa0};
    if (n && type == 1)
        k_width<<<(unsigned)((n + 63) / 64), 64, 0, ix->stream>>>(rev, ix->T, d_C, d_offs, d_lens, d_woff, d_codes, n, (uint32_t *)ix->d_out);
    else if (n)
        k_width0<<<(unsigned)((n + 63) / 64), 64, 0, ix->stream>>>(fwd, ix->T, d_C, d_offs, d_lens, d_woff, d_codes, n, (uint32_t *)ix->d_out);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipMemcpyAsync(width_out, ix->d_out, tot * 4, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    free(woff);
    return 0;
}

extern "C" int hsa_width_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens,
                               const uint8_t *codes, size_t codes_len, uint32_t *width_out)
{
    return width_batch(ix, 1, n, offs, lens, codes, codes_len, width_out);
}

extern "C" int hsa_width0_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens,
                                const uint8_t *codes, size_t codes_len, uint32_t *width_out)
{
    return width_batch(ix, 0, n, offs, lens, codes, codes_len, width_out);
}

// ---------------------------------------------------------------- synthetic genome
// Same stream as hsa_amd/synth.py genome_words(): word w = splitmix64(seed*golden ^ w),
// 32 bases per u64, base j at bits 2j..2j+1; emitted as LSB-first u32 (16 bases).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_synth(uint64_t T, uint64_t seed, uint32_t *out)
{
    uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t nw = (T + 31) / 32;
    if (w >= nw) return;
    uint64_t x = splitmix64((seed * 0x9E3779B97F4A7C15ull) ^ w);
    uint64_t rem = T - w * 32;
    if (rem < 32) x &= (1ull << (2 * rem)) - 1ull;
    uint64_t lo_words = (T + 15) / 16;
    out[2 * w] = (uint32_t)x;
    if (2 * w + 1 < lo_words) out[2 * w + 1] = (uint32_t)(x >> 32);
}

extern "C" int hsa_synth_genome_device(int device, uint64_t T, uint64_t seed, uint32_t *d_code_lsb)
{
    HSA_HIP(hipSetDevice(device));
    uint64_t nw = (T + 31) / 32;
    k_synth<<<(unsigned)((nw + 255) / 256), 256>>>(T, seed, d_code_lsb);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipDeviceSynchronize());
    return 0;
}

// ---------------------------------------------------------------- roofline probe
// Random 64-byte-sector gather over a table as large as the rank index -- the access
// pattern of the rank queries.  Each lane loads `per_sector` x 16 bytes of one
// uniformly random sector per iteration (1: one 16-byte load, what a rank query of
// the 16-character layout issues; 4: the whole sector), 16 waves per CU.  Gives the
// measured ceiling the search kernels' achieved bandwidth (one sector per query) is
// compared with (tools/membench.hip is the stand-alone version).
// PER = 2: four adjacent lanes share one random sector, each loading 16 bytes of it
// (16 sectors per wave load instruction, every byte of each sector used).
template <int PER>
__global__ void __launch_bounds__(256) k_gather(const uint4 *__restrict__ buf, uint64_t nsec, int iters, uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint64_t s = splitmix64((PER == 2 ? gid >> 2 : gid) + 1);
    for (int it = 0; it < iters; ++it) {
        s = splitmix64(s);
        const uint4 *p = buf + (s % nsec) * 4 + (PER == 1 ? (s >> 62) : PER == 2 ? (gid & 3) : 0);
#pragma unroll
        for (int k = 0; k < (PER == 2 ? 1 : PER); ++k) {
            const uint4 v = p[k];
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads live; never true in practice
}

__global__ void k_fill_words(uint32_t *buf, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = (uint32_t)splitmix64(i);
}

extern "C" int hsa_probe_gather(int device, uint64_t table_bytes, int per_sector, double *gbps)
{
    if (per_sector != 1 && per_sector != 2 && per_sector != 4) { hsa_set_error("per_sector must be 1, 2 or 4"); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    HSA_HIP(hipGetDeviceProperties(&prop, device));
    table_bytes &= ~(uint64_t)63;
    if (table_bytes < (1u << 20)) { hsa_set_error("probe table too small"); return HSA_E_ARG; }
    uint4 *buf = nullptr;
    uint32_t *out = nullptr;
    if (hipMalloc(&buf, table_bytes) != hipSuccess) { hsa_set_error("probe: hipMalloc failed"); return HSA_E_MEM; }
    if (hipMalloc(&out, 64) != hipSuccess) { (void)hipFree(buf); hsa_set_error("probe: hipMalloc failed"); return HSA_E_MEM; }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    float ms = 0;
    const uint64_t nsec = table_bytes / 64;
    const unsigned blocks = (unsigned)prop.multiProcessorCount * 4;   // 16 waves per CU
    const int iters = 1000;
    auto launch = [&](int it) {
        if (per_sector == 1) k_gather<1><<<blocks, 256>>>(buf, nsec, it, out);
        else if (per_sector == 2) k_gather<2><<<blocks, 256>>>(buf, nsec, it, out);
        else k_gather<4><<<blocks, 256>>>(buf, nsec, it, out);
    };
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) { rc = HSA_E_HIP; goto done; }
    k_fill_words<<<4096, 256>>>((uint32_t *)buf, table_bytes / 4);
    launch(iters / 4);                                               // warm-up
    (void)hipEventRecord(e0, 0);
    launch(iters);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
        hsa_set_error("probe: kernel failed");
        rc = HSA_E_HIP;
        goto done;
    }
    *gbps = (double)blocks * 256 * iters * 64 / (ms * 1e-3) / 1e9 / (per_sector == 2 ? 4 : 1);   // sectors x 64 B
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(buf); (void)hipFree(out);
    return rc;
}
