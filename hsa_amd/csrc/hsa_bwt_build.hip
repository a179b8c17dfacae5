// hsa_bwt_build.hip -- BWT construction on the device (the index the search reads).
//
// The reference builds its BWT with an incremental CPU construction
// (BWTIncConstructFromPacked, BWTConstruct.c:108; hours for a 3 Gbp text).  Here:
//   1. suffixes are bucketed by their first 4 characters (256 buckets, histogram);
//   2. consecutive buckets are grouped into batches of <= kBatch suffixes; for each
//      batch the suffix positions are selected, keyed by their first 32 characters
//      (64-bit, first character in the top bits, zero = 'A' padding past the end)
//      and radix-sorted (rocPRIM);
//   3. runs of equal keys (suffixes sharing 32 characters, or running off the end)
//      are ordered exactly on the host by direct suffix comparison with the '$'
//      convention (a suffix that ends sorts before any extension of it);
//   4. BWT[row] = text[SA[row]-1], row 0 being the '$' suffix; the '$' row
//      (suffix 0) is dropped from the code string and reported as inverseSa0,
//      exactly the .bwt convention (BWT.c:156-181, BWT.h:61-83).
// Random texts have essentially no 32-character ties; texts with long exact
// repeats would spend their time in step 3 (documented in DESIGN.md).
// Suffix positions are u32 for texts under 2^32 characters and u64 beyond (config 5:
// the 64-bit index of hsa_index_create_device64); the selection of a batch's
// positions scans the text in chunks of 2^31 positions.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "hsa_internal.h"

static const size_t kBatch = (size_t)1 << 29;

__device__ __forceinline__ uint64_t rev2(uint64_t x)
{
    x = (x >> 32) | (x << 32);
    x = ((x & 0xFFFF0000FFFF0000ull) >> 16) | ((x & 0x0000FFFF0000FFFFull) << 16);
    x = ((x & 0xFF00FF00FF00FF00ull) >> 8) | ((x & 0x00FF00FF00FF00FFull) << 8);
    x = ((x & 0xF0F0F0F0F0F0F0F0ull) >> 4) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = ((x & 0xCCCCCCCCCCCCCCCCull) >> 2) | ((x & 0x3333333333333333ull) << 2);
    return x;
}

// 32 characters from position p, first character in the top bits.  The text is
// LSB-first 2-bit (16 per u32) and zero-padded by >= 3 words past its end.
__device__ __forceinline__ uint64_t key32(const uint32_t *__restrict__ t, uint64_t p)
{
    const uint64_t w = p >> 4;
    const uint32_t s = (uint32_t)(p & 15);
    const uint64_t lo = (uint64_t)t[w] | ((uint64_t)t[w + 1] << 32);
    const uint64_t hi = t[w + 2];
    uint64_t x = s ? ((lo >> (2 * s)) | (hi << (64 - 2 * s))) : lo;
    return rev2(x);
}

__device__ __forceinline__ uint32_t char_at(const uint32_t *__restrict__ t, uint64_t p)
{
    return (t[p >> 4] >> (2 * (p & 15))) & 3u;
}

__global__ void k_reverse_text(const uint32_t *src, uint64_t T, uint32_t *dst, uint64_t nwords)
{
    uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint32_t v = 0;
    for (int j = 0; j < 16; ++j) {
        uint64_t p = w * 16 + j;
        if (p < T) v |= char_at(src, T - 1 - p) << (2 * j);
    }
    dst[w] = v;
}

__global__ void k_hist(const uint32_t *t, uint64_t T, unsigned long long *hist, unsigned long long *cnt)
{
    __shared__ unsigned int h[256];
    __shared__ unsigned int c[4];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
    if (threadIdx.x < 4) c[threadIdx.x] = 0;
    __syncthreads();
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < T; p += stride) {
        atomicAdd(&h[key32(t, p) >> 56], 1u);
        atomicAdd(&c[char_at(t, p)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
    if (threadIdx.x < 4 && c[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], (unsigned long long)c[threadIdx.x]);
}

template <typename P> struct InBuckets {
    const uint32_t *t;
    uint32_t lo, hi;
    __device__ bool operator()(P p) const
    {
        const uint32_t b = (uint32_t)(key32(t, p) >> 56);
        return b >= lo && b < hi;
    }
};

template <typename P>
__global__ void k_keys(const uint32_t *t, const P *pos, size_t n, uint64_t *keys)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = key32(t, pos[i]);
}

__global__ void k_tie_flags(const uint64_t *keys, size_t n, uint8_t *flag)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool t = (i > 0 && keys[i] == keys[i - 1]) || (i + 1 < n && keys[i] == keys[i + 1]);
    flag[i] = t ? 1 : 0;
}

// rows [row0, row0+n) of the full (T+1)-row BWT; row = 1 + sorted rank.
// ... and, with sa_out, every sa_int-th suffix-array value (BWTGenerateSaValue's
// samples, BWTConstruct.c:1241-1316: saValue[row / s] = SA[row] for row % s == 0).
template <typename P>
__global__ void k_bwt_chars(const uint32_t *t, const P *sa, size_t n, uint64_t row0, uint8_t *bwt,
                            unsigned long long *isa0, uint32_t *sa_out, uint32_t sa_int)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const P p = sa[i];
    if (sa_out && (row0 + i) % sa_int == 0) sa_out[(row0 + i) / sa_int] = (uint32_t)p;
    if (p == 0) { *isa0 = row0 + i; bwt[row0 + i] = 0; }
    else bwt[row0 + i] = (uint8_t)char_at(t, p - 1);
}

// pack rows != isa0 into LSB-first 2-bit words
__global__ void k_pack(const uint8_t *bwt, uint64_t T, uint64_t isa0, uint32_t *out, uint64_t nwords)
{
    uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint32_t v = 0;
    for (int j = 0; j < 16; ++j) {
        uint64_t q = w * 16 + j;
        if (q >= T) break;
        uint64_t row = q < isa0 ? q : q + 1;
        v |= (uint32_t)bwt[row] << (2 * j);
    }
    out[w] = v;
}

// ---- host-side exact ordering of tied suffixes ('$' < A < C < G < T)
struct HostText {
    std::vector<uint32_t> w;
    uint64_t T;
    inline uint32_t at(uint64_t p) const { return (w[p >> 4] >> (2 * (p & 15))) & 3u; }
    bool less(uint64_t a, uint64_t b) const
    {
        if (a == b) return false;
        for (;;) {
            if (b >= T) return false;     // suffix b ended: b <= a
            if (a >= T) return true;      // a ended first
            uint32_t ca = at(a), cb = at(b);
            if (ca != cb) return ca < cb;
            ++a; ++b;
        }
    }
};

template <typename P>
static int build_one(int device, uint64_t T, const uint32_t *d_text, uint32_t *d_out, uint64_t *isa0_out,
                     uint64_t C[5], uint32_t sa_int = 0, uint32_t *d_sa = nullptr)
{
    (void)device;
    hipStream_t st = 0;
    const uint64_t nwords = (T + 15) / 16;
    unsigned long long *d_hist = nullptr, *d_isa0 = nullptr;
    HSA_HIP(hipMalloc(&d_hist, (256 + 4 + 1) * sizeof(unsigned long long)));
    HSA_HIP(hipMemset(d_hist, 0, (256 + 4 + 1) * sizeof(unsigned long long)));
    d_isa0 = d_hist + 260;
    k_hist<<<2048, 256, 0, st>>>(d_text, T, d_hist, d_hist + 256);
    HSA_HIP(hipGetLastError());
    unsigned long long hist[260];
    HSA_HIP(hipMemcpy(hist, d_hist, sizeof hist, hipMemcpyDeviceToHost));
    C[0] = 0;
    for (int c = 0; c < 4; ++c) C[c + 1] = C[c] + (uint64_t)hist[256 + c];

    uint8_t *d_bwt = nullptr;
    HSA_HIP(hipMalloc(&d_bwt, T + 16));
    // row 0: the '$' suffix, preceded by the last character
    {
        uint32_t last_word = 0;
        HSA_HIP(hipMemcpy(&last_word, d_text + ((T - 1) >> 4), 4, hipMemcpyDeviceToHost));
        uint8_t c0 = (uint8_t)((last_word >> (2 * ((T - 1) & 15))) & 3u);
        HSA_HIP(hipMemcpy(d_bwt, &c0, 1, hipMemcpyHostToDevice));
    }
    size_t maxb = 0;
    for (int b = 0; b < 256; ++b) maxb = std::max(maxb, (size_t)hist[b]);
    const size_t cap = std::max(std::min(kBatch, (size_t)T), maxb);
    P *d_pos = nullptr, *d_pos2 = nullptr;
    uint64_t *d_key = nullptr, *d_key2 = nullptr;
    uint8_t *d_flag = nullptr;
    size_t *d_nsel = nullptr;
    HSA_HIP(hipMalloc(&d_pos, cap * sizeof(P) + 64));
    HSA_HIP(hipMalloc(&d_pos2, cap * sizeof(P) + 64));
    HSA_HIP(hipMalloc(&d_key, cap * 8 + 64));
    HSA_HIP(hipMalloc(&d_key2, cap * 8 + 64));
    HSA_HIP(hipMalloc(&d_flag, cap + 64));
    HSA_HIP(hipMalloc(&d_nsel, 64));
    void *tmp = nullptr;
    size_t tmp_bytes = 0, need = 0;
    HostText host;
    host.T = T;

    uint64_t row = 1;
    int b = 0;
    while (b < 256) {
        size_t n = 0;
        int e = b;
        while (e < 256 && (n + hist[e] <= cap || e == b)) n += hist[e++];
        if (n == 0) { b = e; continue; }
        // 2. select positions with a bucket in [b, e), 2^31 text positions at a time
        InBuckets<P> pred{d_text, (uint32_t)b, (uint32_t)e};
        size_t got = 0;
        for (uint64_t c0 = 0; c0 < T; c0 += (uint64_t)1 << 31) {
            const size_t cn = (size_t)std::min<uint64_t>(T - c0, (uint64_t)1 << 31);
            rocprim::counting_iterator<P> it((P)c0);
            HSA_HIP(rocprim::select(nullptr, need, it, d_pos + got, d_nsel, cn, pred, st));
            if (need > tmp_bytes) { (void)hipFree(tmp); tmp_bytes = need; HSA_HIP(hipMalloc(&tmp, tmp_bytes)); }
            HSA_HIP(rocprim::select(tmp, need, it, d_pos + got, d_nsel, cn, pred, st));
            size_t k = 0;
            HSA_HIP(hipMemcpyAsync(&k, d_nsel, sizeof k, hipMemcpyDeviceToHost, st));
            HSA_HIP(hipStreamSynchronize(st));
            got += k;
        }
        if (got != n) { hsa_set_error("bwt build: selected %zu of %zu suffixes", got, n); return HSA_E_HIP; }
        k_keys<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d_text, d_pos, n, d_key);
        HSA_HIP(hipGetLastError());
        HSA_HIP(rocprim::radix_sort_pairs(nullptr, need, d_key, d_key2, d_pos, d_pos2, n, 0, 64, st));
        if (need > tmp_bytes) { (void)hipFree(tmp); tmp_bytes = need; HSA_HIP(hipMalloc(&tmp, tmp_bytes)); }
        HSA_HIP(rocprim::radix_sort_pairs(tmp, need, d_key, d_key2, d_pos, d_pos2, n, 0, 64, st));
        // 3. ties
        k_tie_flags<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d_key2, n, d_flag);
        HSA_HIP(hipGetLastError());
        uint32_t *const d_rank = reinterpret_cast<uint32_t *>(d_pos);              // d_pos := tied ranks
        rocprim::counting_iterator<uint32_t> rit(0u);
        HSA_HIP(rocprim::select(nullptr, need, rit, d_flag, d_rank, d_nsel, n, st));
        if (need > tmp_bytes) { (void)hipFree(tmp); tmp_bytes = need; HSA_HIP(hipMalloc(&tmp, tmp_bytes)); }
        HSA_HIP(rocprim::select(tmp, need, rit, d_flag, d_rank, d_nsel, n, st));
        size_t nt = 0;
        HSA_HIP(hipMemcpy(&nt, d_nsel, sizeof nt, hipMemcpyDeviceToHost));
        if (nt) {
            if (host.w.empty()) {
                host.w.resize(nwords + 4, 0);
                HSA_HIP(hipMemcpy(host.w.data(), d_text, nwords * 4, hipMemcpyDeviceToHost));
            }
            std::vector<uint32_t> rk(nt);
            HSA_HIP(hipMemcpy(rk.data(), d_rank, nt * 4, hipMemcpyDeviceToHost));
            // gather the tied keys/positions (ranks are sorted ascending)
            std::vector<uint64_t> kk;
            std::vector<P> pp;
            size_t i = 0;
            while (i < nt) {
                size_t j = i;
                while (j + 1 < nt && rk[j + 1] == rk[j] + 1) ++j;
                size_t len = j - i + 1;
                kk.resize(len); pp.resize(len);
                HSA_HIP(hipMemcpy(kk.data(), d_key2 + rk[i], len * 8, hipMemcpyDeviceToHost));
                HSA_HIP(hipMemcpy(pp.data(), d_pos2 + rk[i], len * sizeof(P), hipMemcpyDeviceToHost));
                size_t g = 0;
                while (g < len) {
                    size_t h = g;
                    while (h + 1 < len && kk[h + 1] == kk[g]) ++h;
                    if (h > g)
                        std::sort(pp.begin() + g, pp.begin() + h + 1,
                                  [&](P x, P y) { return host.less(x, y); });
                    g = h + 1;
                }
                HSA_HIP(hipMemcpy(d_pos2 + rk[i], pp.data(), len * sizeof(P), hipMemcpyHostToDevice));
                i = j + 1;
            }
        }
        // 4. BWT characters of these rows
        k_bwt_chars<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d_text, d_pos2, n, row, d_bwt, d_isa0, d_sa, sa_int);
        HSA_HIP(hipGetLastError());
        row += n;
        b = e;
    }
    HSA_HIP(hipDeviceSynchronize());
    unsigned long long isa0 = 0;
    HSA_HIP(hipMemcpy(&isa0, d_isa0, 8, hipMemcpyDeviceToHost));
    k_pack<<<(unsigned)((nwords + 255) / 256), 256, 0, st>>>(d_bwt, T, isa0, d_out, nwords);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipDeviceSynchronize());
    *isa0_out = (uint64_t)isa0;
    (void)hipFree(tmp); (void)hipFree(d_pos); (void)hipFree(d_pos2); (void)hipFree(d_key); (void)hipFree(d_key2);
    (void)hipFree(d_flag); (void)hipFree(d_nsel); (void)hipFree(d_bwt); (void)hipFree(d_hist);
    return 0;
}

static int build_bwt(int device, uint64_t T, const uint32_t *d_text_lsb, int reverse, uint32_t *d_bwt_lsb,
                     uint64_t *isa0, uint64_t C[5], uint32_t sa_int = 0, uint32_t *d_sa = nullptr)
{
    if (T == 0) { hsa_set_error("empty text"); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(device));
    const uint64_t nwords = (T + 15) / 16;
    uint32_t *t = nullptr;
    HSA_HIP(hipMalloc(&t, (nwords + 8) * 4));
    HSA_HIP(hipMemset(t, 0, (nwords + 8) * 4));
    if (reverse) {
        k_reverse_text<<<(unsigned)((nwords + 255) / 256), 256>>>(d_text_lsb, T, t, nwords);
        HSA_HIP(hipGetLastError());
    } else {
        HSA_HIP(hipMemcpy(t, d_text_lsb, nwords * 4, hipMemcpyDeviceToDevice));
        if (T & 15) {   // clear the tail of the last word
            uint32_t last;
            HSA_HIP(hipMemcpy(&last, t + nwords - 1, 4, hipMemcpyDeviceToHost));
            last &= (1u << (2 * (T & 15))) - 1u;
            HSA_HIP(hipMemcpy(t + nwords - 1, &last, 4, hipMemcpyHostToDevice));
        }
    }
    // u32 suffix positions while they fit (half the sort traffic of u64)
    int rc = T < 0xFFFFFFFFull ? build_one<uint32_t>(device, T, t, d_bwt_lsb, isa0, C, sa_int, d_sa)
                               : build_one<uint64_t>(device, T, t, d_bwt_lsb, isa0, C, sa_int, d_sa);
    (void)hipFree(t);
    return rc;
}

extern "C" int hsa_build_bwt_device64(int device, uint64_t T, const uint32_t *d_text_lsb, int reverse,
                                      uint32_t *d_bwt_lsb, uint64_t *isa0, uint64_t C[5])
{
    return build_bwt(device, T, d_text_lsb, reverse, d_bwt_lsb, isa0, C);
}

// The BWT of the text as given plus its sampled suffix array (hsa_amd/index_build.py:
// the .sa file of `HSA index`, whose values are u32, BWTConstruct.c:1373-1392).  SA
// samples rows 1, 2, ... of every sa_interval-th row go to d_sa[row / sa_interval];
// d_sa[0] (the '$' row, SA = T) is the caller's.
extern "C" int hsa_build_bwt_index_device(int device, uint64_t T, const uint32_t *d_text_lsb, uint32_t *d_bwt_lsb,
                                          uint64_t *isa0, uint64_t C[5], uint32_t sa_interval, uint32_t *d_sa)
{
    if (T == 0 || T >= 0xFFFFFFFFull) { hsa_set_error("text length must be in [1, 2^32-1) (u32 SA values)"); return HSA_E_ARG; }
    if (d_sa && sa_interval == 0) { hsa_set_error("sa_interval must be > 0"); return HSA_E_ARG; }
    return build_bwt(device, T, d_text_lsb, 0, d_bwt_lsb, isa0, C, sa_interval, d_sa);
}

// The 32-bit entry point: the .bwt header fields are u32 (BWT.h:61-83)
extern "C" int hsa_build_bwt_device(int device, uint64_t T, const uint32_t *d_text_lsb, int reverse,
                                    uint32_t *d_bwt_lsb, uint32_t *isa0, uint32_t C[5])
{
    if (T == 0 || T >= 0xFFFFFFFFull) {
        hsa_set_error("text length must be in [1, 2^32-1) (hsa_build_bwt_device64 builds longer ones)");
        return HSA_E_ARG;
    }
    uint64_t i64 = 0, c64[5] = {0, 0, 0, 0, 0};
    const int rc = build_bwt(device, T, d_text_lsb, reverse, d_bwt_lsb, &i64, c64);
    if (rc) return rc;
    *isa0 = (uint32_t)i64;
    for (int c = 0; c < 5; ++c) C[c] = (uint32_t)c64[c];
    return 0;
}
