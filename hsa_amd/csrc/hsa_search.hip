// hsa_search.hip -- the 32-bit search API (include/hsa_gpu.h): host-array and
// device-resident batches, direct bwt_match_gap calls, the splice seeds; the kernels
// are in hsa_search_kernels.h.
#include "hsa_search_kernels.h"

#include <vector>

// ---------------------------------------------------------------- splice seeds
// The seed calls of bwt_splice_match (bwtgap.c:797-812) for every read the main pass
// flagged HSA_F_FALLBACK: one thread per (read, strand).  The strand's three seeds
// t = 0, 1, 2 (sl = len / 3, la_t = sl + (t == 2 ? len % 3 : 0)) search [t sl, t sl +
// la_t) of the strand sequence with the widths of its PREFIX of length la_t
// (bwtgap.c:807-809; bwt_cal_width type 1, bwtaln.c:84-97: forward extension on the
// reverse BWT).  The three prefixes share their first sl positions, so one chain over
// la_2 characters fills all three width slots; each slot ends with its own terminal
// {0, bid + 1} (bwtaln.c:113-114).
struct SeedArgs {
    RankDir rev;
    uint32_t T;
    uint32_t C[5];
    const hsa_job_t *rjobs;
    const uint8_t *rcodes;
    const uint32_t *rflags;
    uint32_t n_reads;
    int32_t max_seed_diff;
    uint32_t code_stride, pair_stride;   // per read: seed codes (bytes), width pairs
    hsa_job_t *jobs;
    hsa_mg_job_t *mg;
    uint8_t *codes;
    int32_t *cw;
    int32_t *list;
    unsigned long long *count;
    unsigned long long *ctr;
};

__global__ void __launch_bounds__(BLOCK) k_seed_prep(SeedArgs a)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t r = t >> 1, s = t & 1u;
    if (r >= a.n_reads || !(a.rflags[r] & HSA_F_FALLBACK)) return;
    const hsa_job_t R = a.rjobs[r];
    const uint32_t L = R.len, sl = L / 3u;
    if (sl < 1) return;
    const uint32_t la2 = sl + L % 3u;
    auto base = [&](uint32_t p) -> uint32_t {          // strand s, position p
        const uint32_t c = a.rcodes[R.off + (s ? L - 1u - p : p)];
        return s && c < 4 ? 3u - c : c;
    };
    // call i = 3 s + tt of read r: codes and width pairs at fixed offsets in the read's slots
    uint32_t coff[3], poff[3], la[3];
    {
        uint32_t co = 0, po = 0;
        for (uint32_t i = 0; i < 6; ++i) {
            const uint32_t l_i = sl + (i % 3 == 2 ? L % 3u : 0u);
            if (i / 3 == s) { coff[i % 3] = co; poff[i % 3] = po; la[i % 3] = l_i; }
            co += l_i; po += l_i + 1;
        }
    }
    uint8_t *const cbase = a.codes + (size_t)r * a.code_stride;
    int32_t *const wbase = a.cw + 2 * (size_t)r * a.pair_stride;
    uint32_t k = 0, l = a.T, bid = 0, bid_sl = 0, q = 0;
    for (uint32_t p = 0; p < la2; ++p) {
        const uint32_t c = base(p);
        if (c < 4) {
            uint32_t ok, ol;
            hsa_occ1_pair(a.rev, k, l + 1u, c, ok, ol);
            q += 2;
            const uint32_t cc = c == 0 ? a.C[0] : c == 1 ? a.C[1] : c == 2 ? a.C[2] : a.C[3];
            k = cc + ok + 1u;
            l = cc + ol;
        }
        if (k > l || c > 3) { k = 0; l = a.T; ++bid; }
        const int32_t w = (int32_t)(l - k + 1u);
        for (uint32_t tt = 0; tt < 3; ++tt)
            if (p < la[tt]) { wbase[2 * (poff[tt] + p)] = w; wbase[2 * (poff[tt] + p) + 1] = (int32_t)bid; }
        if (p + 1 == sl) bid_sl = bid;
        // seed codes: strand position p belongs to seed tt = p / sl (the last seed runs to la2 + 2 sl)
    }
    for (uint32_t tt = 0; tt < 3; ++tt) {
        const uint32_t term_bid = (la[tt] == sl ? bid_sl : bid) + 1u;
        wbase[2 * (poff[tt] + la[tt])] = 0;
        wbase[2 * (poff[tt] + la[tt]) + 1] = (int32_t)term_bid;
        for (uint32_t p = 0; p < la[tt]; ++p) cbase[coff[tt] + p] = (uint8_t)base(tt * sl + p);
        const uint32_t j = r * 6u + 3u * s + tt;
        hsa_job_t J;
        J.off = (uint64_t)r * a.code_stride + coff[tt];
        J.len = la[tt];
        J.max_diff = a.max_seed_diff;
        J.seed_len = (int32_t)la[tt];
        J.regime = 0;
        a.jobs[j] = J;
        hsa_mg_job_t M;
        M.wb_off = (uint64_t)r * a.pair_stride + poff[tt];
        M.ws_off = 0;
        M.strand = (int32_t)s;
        M.seed = HSA_SEED_ALIAS;
        a.mg[j] = M;
    }
    const unsigned long long b0 = atomicAdd(a.count, 3ull);
    for (uint32_t tt = 0; tt < 3; ++tt) a.list[b0 + tt] = (int32_t)(r * 6u + 3u * s + tt);
    atomicAdd(&a.ctr[7], (unsigned long long)q);
}

// ---------------------------------------------------------------- host side
#ifdef HSA_DIAG
extern "C" int hsa_diag_read(unsigned long long *out, int n_blocks)
{
    HSA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * 4 * (size_t)n_blocks));
    return 0;
}
extern "C" int hsa_diag_counters(unsigned long long *out, int reset)
{
    HSA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dctr), sizeof(unsigned long long) * 32));
    if (reset) {
        unsigned long long z[32] = {0};
        HSA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dctr), z, sizeof z));
    }
    return 0;
}
#endif
struct MgHost {
    const hsa_mg_job_t *mg;
    const int32_t *widths;
    size_t width_pairs;
    int32_t *widths_out;
};

// Checks of a caller-width batch; max_seed = the longest own width_seed.  A width_seed
// with seed_len > len makes the reference read outside it: refused.
static int mg_limits(const hsa_job_t *jobs, const hsa_mg_job_t *mg, int n, const MgHost &mh, int &max_seed)
{
    max_seed = 0;
    for (int j = 0; j < n; ++j) {
        const hsa_mg_job_t &M = mg[j];
        const uint32_t len = jobs[j].len;
        if (M.strand != 0 && M.strand != 1) { hsa_set_error("call %d: strand %d", j, M.strand); return HSA_E_ARG; }
        if (M.seed < HSA_SEED_NONE || M.seed > HSA_SEED_ALIAS) { hsa_set_error("call %d: seed kind", j); return HSA_E_ARG; }
        if (M.seed != HSA_SEED_NONE && (jobs[j].seed_len < 0 || jobs[j].seed_len > (int)len)) {
            hsa_set_error("call %d: width_seed with seed_len %d outside [0, len %u] (undefined in the reference)", j,
                          jobs[j].seed_len, len);
            return HSA_E_ARG;
        }
        if (M.wb_off + len + 1 > mh.width_pairs ||
            (M.seed == HSA_SEED_OWN && M.ws_off + (uint64_t)jobs[j].seed_len + 1 > mh.width_pairs)) {
            hsa_set_error("call %d: widths outside the width array", j);
            return HSA_E_ARG;
        }
        for (uint32_t t = 0; t <= len; ++t)
            if (mh.widths[2 * (M.wb_off + t) + 1] < 0) { hsa_set_error("call %d: negative bid", j); return HSA_E_ARG; }
        if (M.seed == HSA_SEED_OWN) {
            for (int t = 0; t <= jobs[j].seed_len; ++t)
                if (mh.widths[2 * (M.ws_off + t) + 1] < 0) { hsa_set_error("call %d: negative bid", j); return HSA_E_ARG; }
            if (jobs[j].seed_len > max_seed) max_seed = jobs[j].seed_len;
        }
    }
    return 0;
}

// k_search_any over host arrays (hsa_search_any.h): reads longer than k_search holds,
// or every read of a regime outside its layouts.  Same outputs as search_batch_impl.
static long search_any_host(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs, int n,
                            const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                            uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh)
{
    hipStream_t st = ix->stream;
    uint32_t max_len = 1, max_seed = 0;
    for (int j = 0; j < n; ++j) {
        if (jobs[j].len > max_len) max_len = jobs[j].len;
        const bool own = mh ? mh->mg[j].seed == HSA_SEED_OWN : (int)jobs[j].len > jobs[j].seed_len;
        if (own && (uint32_t)jobs[j].seed_len > max_seed) max_seed = (uint32_t)jobs[j].seed_len;
    }
    AnyBufs AB;
    int rc = any_prepare(ix, regimes, n_regimes, (size_t)n, st, AB);
    if (rc) return rc;
    // inputs after the fast path's regime staging ([0, 1536) of d_in stays as it is)
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_jobs = 1536, o_codes = o_jobs + al((size_t)n * sizeof(hsa_job_t));
    const size_t o_mg = o_codes + al(codes_len + 64), o_cw = o_mg + (mh ? al((size_t)n * sizeof(hsa_mg_job_t)) : 0);
    const size_t cw_bytes = mh ? mh->width_pairs * 8 : 0;
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, o_cw + cw_bytes + 256))) return rc;
    if (before != ix->d_in) ix->staged_valid = 0;       // the regime staging went with the old buffer
    char *din = (char *)ix->d_in;
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, sizeof(hsa_job_t) * n, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    MgPass mgp{nullptr, nullptr};
    if (mh) {
        HSA_HIP(hipMemcpyAsync(din + o_mg, mh->mg, sizeof(hsa_mg_job_t) * n, hipMemcpyHostToDevice, st));
        HSA_HIP(hipMemcpyAsync(din + o_cw, mh->widths, cw_bytes, hipMemcpyHostToDevice, st));
        mgp = MgPass{(const hsa_mg_job_t *)(din + o_mg), (int32_t *)(din + o_cw)};
    }
    const uint64_t hit_cap = (uint64_t)n * 64 + 65536;
    const size_t o_fl = al((size_t)n * 4), o_ho = o_fl + al((size_t)n * 4), o_hits = o_ho + al((size_t)n * 8);
    if ((rc = hsa_grow(&ix->d_out, &ix->d_out_cap, o_hits + hit_cap * 36 + 256))) return rc;
    char *dout = (char *)ix->d_out;
    unsigned long long *d_ctr = (unsigned long long *)ix->d_ctr;
    HSA_HIP(hipMemsetAsync(d_ctr, 0, 16 * sizeof(unsigned long long), st));
    HSA_HIP(hipEventRecord(ix->ev0, st));
    const hsa_job_t *dj = (const hsa_job_t *)(din + o_jobs);
    const uint8_t *dc = (const uint8_t *)(din + o_codes);
    int32_t *d_n = (int32_t *)dout;
    uint32_t *d_fl = (uint32_t *)(dout + o_fl);
    uint64_t *d_ho = (uint64_t *)(dout + o_ho);
    uint32_t *d_hits = (uint32_t *)(dout + o_hits);
    if ((rc = any_pass<uint32_t>(ix, AB, regimes, n_regimes, dj, nullptr, nullptr, n, (size_t)n, max_len, max_seed, dc,
                                 mh ? &mgp : nullptr, d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, AB.cnt + 2, AB.l_ovf,
                                 AB.cnt + 3, false, st)) ||
        (rc = any_pass<uint32_t>(ix, AB, regimes, n_regimes, dj, AB.l_ovf, AB.cnt + 3, 0, (size_t)n, max_len, max_seed,
                                 dc, mh ? &mgp : nullptr, d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, AB.cnt + 4, nullptr,
                                 nullptr, true, st)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    unsigned long long ctr[16];
    HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(n_aln, d_n, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(flags, d_fl, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(hit_off, d_ho, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    if (ctr[5]) { hsa_set_error("%llu reads pushed a score past the regime's n_stacks", ctr[5]); return HSA_E_ARG; }
    if (ctr[11]) { hsa_set_error("%llu reads exceed the large-pass capacity", ctr[11]); return HSA_E_ARG; }
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    const uint64_t total = ctr[1];
    uint32_t *h = (uint32_t *)malloc((total + 1) * 36);
    if (total) HSA_HIP(hipMemcpy(h, d_hits, total * 36, hipMemcpyDeviceToHost));
    if (mh) {
        int32_t *cw = (int32_t *)malloc(cw_bytes + 8);
        HSA_HIP(hipMemcpy(cw, din + o_cw, cw_bytes, hipMemcpyDeviceToHost));
        for (int j = 0; j < n; ++j)
            memcpy(mh->widths_out + 2 * mh->mg[j].wb_off, cw + 2 * mh->mg[j].wb_off, 8 * ((size_t)jobs[j].len + 1));
        free(cw);
    }
    if (stats) {
        stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
        stats->kernel_ms += ms; stats->main_kernel_ms += ms; stats->main_launches += 1;
    }
    *hits_out = h;
    return (long)total;
}

// A batch with reads (or a regime) k_search cannot hold: the reads it can hold through
// search_batch_impl, the others through k_search_any; outputs merged in job order.
static long search_batch_impl(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                              int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                              uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh);

static long search_split(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs, int n,
                         const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                         uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh, bool fast_rg)
{
    std::vector<int> part[2];                        // 0: k_search, 1: k_search_any
    for (int j = 0; j < n; ++j) part[fast_rg && jobs[j].len <= FAST_MAX_LEN ? 0 : 1].push_back(j);
    uint32_t *hs[2] = {nullptr, nullptr};
    long tot[2] = {0, 0};
    if (stats) memset(stats, 0, sizeof *stats);
    for (int k = 0; k < 2; ++k) {
        const int m = (int)part[k].size();
        if (m == 0) continue;
        std::vector<hsa_job_t> pj(m);
        std::vector<hsa_mg_job_t> pm(mh ? m : 0);
        for (int q = 0; q < m; ++q) {
            pj[q] = jobs[part[k][q]];
            if (mh) pm[q] = mh->mg[part[k][q]];
        }
        const MgHost pmh = mh ? MgHost{pm.data(), mh->widths, mh->width_pairs, mh->widths_out} : MgHost{};
        std::vector<int32_t> na(m);
        std::vector<uint32_t> fl(m);
        std::vector<uint64_t> ho(m);
        hsa_stats_t ps;
        memset(&ps, 0, sizeof ps);
        const long t = k == 0 ? search_batch_impl(ix, regimes, n_regimes, pj.data(), m, codes, codes_len, na.data(), fl.data(),
                                                  ho.data(), &hs[k], &ps, mh ? &pmh : nullptr)
                              : search_any_host(ix, regimes, n_regimes, pj.data(), m, codes, codes_len, na.data(),
                                                fl.data(), ho.data(), &hs[k], &ps, mh ? &pmh : nullptr);
        if (t < 0) { free(hs[0]); free(hs[1]); return t; }
        tot[k] = t;
        for (int q = 0; q < m; ++q) {
            const int j = part[k][q];
            n_aln[j] = na[q]; flags[j] = fl[q]; hit_off[j] = ho[q] + (k ? (uint64_t)tot[0] : 0);
        }
        if (stats) {
            stats->rank_queries += ps.rank_queries; stats->blocks_loaded += ps.blocks_loaded; stats->pops += ps.pops;
            stats->overflow_reruns += ps.overflow_reruns; stats->kernel_ms += ps.kernel_ms;
            stats->main_kernel_ms += ps.main_kernel_ms; stats->main_launches += ps.main_launches;
        }
    }
    uint32_t *h = (uint32_t *)malloc(((size_t)tot[0] + (size_t)tot[1] + 1) * 36);
    if (tot[0]) memcpy(h, hs[0], (size_t)tot[0] * 36);
    if (tot[1]) memcpy(h + (size_t)tot[0] * 9, hs[1], (size_t)tot[1] * 36);
    free(hs[0]); free(hs[1]);
    *hits_out = h;
    return tot[0] + tot[1];
}

static long search_batch_impl(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                              int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                              uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh)
{
    *hits_out = nullptr;
    if (n_regimes < 1 || n_regimes > 2) { hsa_set_error("1 or 2 regimes"); return HSA_E_ARG; }
    if (int rc0 = hsa_need32(ix)) return rc0;
    int rc = check_regimes(regimes, n_regimes);
    if (rc) return rc;
    int max_len, max_seed;
    if ((rc = jobs_limits(jobs, n_jobs, max_len, max_seed))) return rc;
    if (mh && (rc = mg_limits(jobs, mh->mg, n_jobs, *mh, max_seed))) return rc;
    if (codes_len >= 0xFFFFFFFFull) { hsa_set_error("read codes of one call must be < 4 GiB"); return HSA_E_ARG; }
    for (int j = 0; j < n_jobs; ++j)        // the kernels read codes[off, off + len) of every job
        if (jobs[j].off > codes_len || jobs[j].len > codes_len - jobs[j].off) {
            hsa_set_error("job %d: codes [%llu, +%u) past codes_len %zu", j, (unsigned long long)jobs[j].off,
                          jobs[j].len, codes_len);
            return HSA_E_ARG;
        }
    {
        const bool fast_rg = fast_regimes(regimes, n_regimes);
        bool all_fit = fast_rg;
        for (int j = 0; j < n_jobs && all_fit; ++j) all_fit = jobs[j].len <= FAST_MAX_LEN;
        if (!all_fit)
            return search_split(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off, hits_out,
                                stats, mh, fast_rg);
    }
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = ix->stream;
    if (stats) memset(stats, 0, sizeof *stats);
    if (n_jobs == 0) { *hits_out = (uint32_t *)calloc(9, 4); return 0; }
    static const bool verbose = getenv("HSA_VERBOSE") != nullptr;
    const auto now = []() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; };
    const double tv0 = verbose ? now() : 0.0;

    // device staging: regimes+bmap | jobs | list | codes [| mg jobs | caller widths]
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_reg = 0, o_jobs = 1536, o_list = o_jobs + al((size_t)n_jobs * sizeof(hsa_job_t));
    const size_t o_codes = o_list + al((size_t)n_jobs * 4);
    const size_t o_mg = o_codes + al(codes_len + 1);
    const size_t o_cw = o_mg + (mh ? al((size_t)n_jobs * sizeof(hsa_mg_job_t)) : 0);
    const size_t cw_bytes = mh ? mh->width_pairs * 8 : 0;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, o_cw + cw_bytes + 256))) return rc;
    char *din = (char *)ix->d_in;
    int nb = 0;
    if ((rc = stage_regimes(ix, regimes, n_regimes, din + o_reg, nb, st, true))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)(din + o_reg);
    const uint8_t *d_bmap = (const uint8_t *)(din + o_reg + 256);
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, sizeof(hsa_job_t) * n_jobs, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    MgPass mgp{nullptr, nullptr};
    if (mh) {
        HSA_HIP(hipMemcpyAsync(din + o_mg, mh->mg, sizeof(hsa_mg_job_t) * n_jobs, hipMemcpyHostToDevice, st));
        HSA_HIP(hipMemcpyAsync(din + o_cw, mh->widths, cw_bytes, hipMemcpyHostToDevice, st));
        mgp = MgPass{(const hsa_mg_job_t *)(din + o_mg), (int32_t *)(din + o_cw)};
    }
    const MgPass *mgpp = mh ? &mgp : nullptr;
    // outputs: n_aln | flags | hit_off | hits
    uint64_t hit_cap = (uint64_t)n_jobs * 4 + 4096;
    const size_t o_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_ho = o_fl + ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_hits = o_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
    if ((rc = hsa_grow(&ix->d_out, &ix->d_out_cap, o_hits + hit_cap * 36 + 256))) return rc;
    char *dout = (char *)ix->d_out;
    int32_t *d_n = (int32_t *)dout;
    uint32_t *d_fl = (uint32_t *)(dout + o_fl);
    uint64_t *d_ho = (uint64_t *)(dout + o_ho);
    uint32_t *d_hits = (uint32_t *)(dout + o_hits);
    unsigned long long *d_ctr = (unsigned long long *)ix->d_ctr;

    LaunchPlan P;
    const bool gaps = any_gaps(regimes, n_regimes);
    const bool wide = need_wide(regimes, n_regimes);
    bool nib_ok = !mgpp && nib_exact(regimes, n_regimes);
    for (int j = 0; j < n_jobs && nib_ok; ++j) nib_ok = jobs[j].max_diff <= 6;
    if ((rc = plan_launch(ix, n_jobs, max_len, max_seed, nb, gaps, wide, PASS_MAIN, P, 0, 16, nib_ok))) return rc;
    HSA_HIP(hipEventRecord(ix->ev0, st));
    if ((rc = launch_pass(ix, P, ix->main, d_reg, d_bmap, (const hsa_job_t *)(din + o_jobs), nullptr, n_jobs,
                          max_len, max_seed, (const uint8_t *)(din + o_codes), d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, st,
                          nullptr, nullptr, 0, mgpp)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    unsigned long long ctr[8];
    HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(n_aln, d_n, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(flags, d_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(hit_off, d_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    if (ctr[5]) { hsa_set_error("%llu reads exceed the regime's max_diff bound", ctr[5]); return HSA_E_ARG; }
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    uint64_t total = ctr[1] < hit_cap ? ctr[1] : hit_cap;
    const double tv1 = verbose ? now() : 0.0;
    uint32_t *h = (uint32_t *)malloc((total + 1) * 36);
    if (total) HSA_HIP(hipMemcpy(h, d_hits, total * 36, hipMemcpyDeviceToHost));
    if (verbose)
        fprintf(stderr, "[hsa] search of %d reads: copies in + kernels + result arrays out %.1f ms (kernels %.1f ms), "
                        "hits out %.1f ms\n", n_jobs, 1e3 * (tv1 - tv0), ms, 1e3 * (now() - tv1));
    if (stats) {
        stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
        stats->kernel_ms += ms; stats->main_kernel_ms += ms; stats->main_launches += 1;
    }

    // overflowed reads: re-run with large per-read capacity (never a CPU path)
    for (int round = 0; round < 4; ++round) {
        int32_t *list = (int32_t *)malloc(sizeof(int32_t) * n_jobs);
        int n_over = 0;
        for (int j = 0; j < n_jobs; ++j) if (flags[j] & HSA_F_OVERFLOW) list[n_over++] = j;
        if (n_over == 0) { free(list); break; }
        if (stats) stats->overflow_reruns += n_over;
        LaunchPlan B;
        int max_entries = 0;
        for (int r = 0; r < n_regimes; ++r) max_entries = regimes[r].max_entries > max_entries ? regimes[r].max_entries : max_entries;
        const int mode = round == 0 ? PASS_BIG : PASS_HUGE;
        if ((rc = plan_launch(ix, n_over, max_len, max_seed, nb, gaps, wide, mode, B, max_entries, 16, nib_ok))) {
            free(list); free(h); return rc;
        }
        uint64_t cap2 = (uint64_t)n_over * 256 * (round + 1) + 65536;
        void *d2 = nullptr;
        size_t o2_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
        size_t o2_ho = o2_fl * 2, o2_hits = o2_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
        HSA_HIP(hipMalloc(&d2, o2_hits + cap2 * 36));
        HSA_HIP(hipMemcpyAsync(din + o_list, list, sizeof(int32_t) * n_over, hipMemcpyHostToDevice, st));
        char *c2 = (char *)d2;
        HSA_HIP(hipEventRecord(ix->ev0, st));
        if ((rc = launch_pass(ix, B, mode == PASS_BIG ? ix->big : ix->huge, d_reg, d_bmap, (const hsa_job_t *)(din + o_jobs),
                              (const int32_t *)(din + o_list), n_over, max_len, max_seed,
                              (const uint8_t *)(din + o_codes), (int32_t *)c2,
                              (uint32_t *)(c2 + o2_fl), (uint64_t *)(c2 + o2_ho), (uint32_t *)(c2 + o2_hits), cap2,
                              d_ctr, st, nullptr, nullptr, 0, mgpp))) {
            free(list); free(h); (void)hipFree(d2); return rc;
        }
        HSA_HIP(hipEventRecord(ix->ev1, st));
        int32_t *n2 = (int32_t *)malloc((size_t)n_jobs * 4);
        uint32_t *f2 = (uint32_t *)malloc((size_t)n_jobs * 4);
        uint64_t *o2 = (uint64_t *)malloc((size_t)n_jobs * 8);
        HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(n2, c2, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(f2, c2 + o2_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(o2, c2 + o2_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipStreamSynchronize(st));
        HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
        uint64_t t2 = ctr[1] < cap2 ? ctr[1] : cap2;
        h = (uint32_t *)realloc(h, (total + t2 + 1) * 36);
        if (t2) HSA_HIP(hipMemcpy(h + total * 9, c2 + o2_hits, t2 * 36, hipMemcpyDeviceToHost));
        for (int q = 0; q < n_over; ++q) {
            int j = list[q];
            n_aln[j] = n2[j]; flags[j] = f2[j]; hit_off[j] = o2[j] + total;
        }
        total += t2;
        if (stats) {
            stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
            stats->kernel_ms += ms;
        }
        free(n2); free(f2); free(o2); free(list);
        (void)hipFree(d2);
    }
    for (int j = 0; j < n_jobs; ++j)
        if (flags[j] & HSA_F_OVERFLOW) { hsa_set_error("read %d exceeds the large-pass capacity", j); free(h); return HSA_E_ARG; }
    if (mh) {
        // width_back of every call after its search (k_widths_export wrote them in place)
        int32_t *cw = (int32_t *)malloc(cw_bytes + 8);
        HSA_HIP(hipMemcpy(cw, din + o_cw, cw_bytes, hipMemcpyDeviceToHost));
        for (int j = 0; j < n_jobs; ++j)
            memcpy(mh->widths_out + 2 * mh->mg[j].wb_off, cw + 2 * mh->mg[j].wb_off, 8 * ((size_t)jobs[j].len + 1));
        free(cw);
    }
    *hits_out = h;
    return (long)total;
}

extern "C" long hsa_search_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                                 int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                                 uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats)
{
    return search_batch_impl(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off, hits_out,
                             stats, nullptr);
}

extern "C" long hsa_match_gap_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                                    const hsa_mg_job_t *mg, int n_jobs, const uint8_t *codes, size_t codes_len,
                                    const int32_t *widths, size_t width_pairs, int32_t *widths_out, int32_t *n_aln,
                                    uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats)
{
    *hits_out = nullptr;
    if (n_jobs > 0 && (!mg || !widths || !widths_out)) { hsa_set_error("hsa_match_gap_batch: null argument"); return HSA_E_ARG; }
    uint32_t *flags = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)n_jobs + 1));
    const MgHost mh{mg, widths, width_pairs, widths_out};
    const long r = search_batch_impl(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off,
                                     hits_out, stats, &mh);
    free(flags);
    return r;
}

extern "C" int hsa_search_device(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                                 const hsa_device_batch_t *b, void *stream)
{
    if (int rc = hsa_need32(ix)) return rc;
    return search_device_impl<uint32_t>(ix, regimes, n_regimes, b, stream);
}

extern "C" int hsa_splice_seeds_device(hsa_index_t *ix, const hsa_regime_t *seed_regime, const hsa_seed_batch_t *b,
                                       void *stream)
{
    if (int rc0 = hsa_need32(ix)) return rc0;
    int rc = check_regimes(seed_regime, 1);
    if (rc) return rc;
    if (seed_regime->max_gapo != 0) { hsa_set_error("seed searches have no gap opens (bwtgap.c:772)"); return HSA_E_ARG; }
    if (b->max_len < 3 || b->max_len > 1023 || b->n_jobs < 0) { hsa_set_error("max_len/n_jobs out of range"); return HSA_E_ARG; }
    const size_t n = (size_t)b->n_jobs, calls = 6 * n;
    if (n == 0) return 0;
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    const uint32_t code_stride = (uint32_t)(2 * b->max_len), pair_stride = (uint32_t)(2 * b->max_len + 6);
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_mg = al(calls * sizeof(hsa_job_t)), o_list = o_mg + al(calls * sizeof(hsa_mg_job_t));
    const size_t o_fl = o_list + al(calls * 4), o_cnt = o_fl + al(calls * 4), o_codes = o_cnt + 256;
    const size_t o_cw = o_codes + al(n * code_stride), total = o_cw + n * pair_stride * 8 + 256;
    if ((rc = hsa_grow(&ix->d_seed, &ix->d_seed_cap, total))) return rc;
    char *d = (char *)ix->d_seed;
    unsigned long long *cnt = (unsigned long long *)(d + o_cnt);
    unsigned long long *ctr = (unsigned long long *)b->d_counters;
    HSA_HIP(hipMemsetAsync(cnt, 0, 8, st));
    SeedArgs S;
    S.rev = RankDir{ix->blk[1], ix->risa0};
    S.T = ix->T;
    memcpy(S.C, ix->C, sizeof S.C);
    S.rjobs = b->d_jobs; S.rcodes = b->d_codes; S.rflags = b->d_flags; S.n_reads = (uint32_t)n;
    S.max_seed_diff = seed_regime->max_diff;
    S.code_stride = code_stride; S.pair_stride = pair_stride;
    S.jobs = (hsa_job_t *)d; S.mg = (hsa_mg_job_t *)(d + o_mg); S.codes = (uint8_t *)(d + o_codes);
    S.cw = (int32_t *)(d + o_cw); S.list = (int32_t *)(d + o_list); S.count = cnt; S.ctr = ctr;
    // the search pass zeroes the counters first; the width queries are added after it
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1536))) return rc;
    int nb = 0;
    if ((rc = stage_regimes(ix, seed_regime, 1, (char *)ix->d_in, nb, st, before != ix->d_in))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)ix->d_in;
    const uint8_t *d_bmap = (const uint8_t *)ix->d_in + 256;
    const int seed_max = b->max_len / 3 + 2;
    LaunchPlan P, B, H;
    const bool wide = need_wide(seed_regime, 1);
    if ((rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_MAIN, P)) ||
        (rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_BIG, B)) ||
        (rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_HUGE, H, seed_regime->max_entries)))
        return rc;
    if ((rc = hsa_grow(&ix->d_ovf, &ix->d_ovf_cap, calls * 4 + 64)) ||
        (rc = hsa_grow(&ix->d_ovf2, &ix->d_ovf2_cap, calls * 4 + 64)))
        return rc;
    HSA_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_seed_prep, dim3((unsigned)((2 * n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, S);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipEventRecord(ix->ev0, st));
    const MgPass mgp{S.mg, S.cw};
    uint32_t *sfl = (uint32_t *)(d + o_fl);
    // qctr 10: the pass's queue head, so that counter [7] (width queries) survives
    if ((rc = launch_pass(ix, P, ix->main, d_reg, d_bmap, S.jobs, S.list, (int)calls, seed_max, 0, S.codes,
                          b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, (int32_t *)ix->d_ovf, cnt, 10,
                          &mgp)))
        return rc;
    if ((rc = launch_pass(ix, B, ix->big, d_reg, d_bmap, S.jobs, (const int32_t *)ix->d_ovf, (int)calls, seed_max, 0,
                          S.codes, b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, (int32_t *)ix->d_ovf2,
                          ctr + 8, 9, &mgp, 12)) ||
        (rc = launch_pass(ix, H, ix->huge, d_reg, d_bmap, S.jobs, (const int32_t *)ix->d_ovf2, (int)calls, seed_max, 0,
                          S.codes, b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, nullptr, ctr + 12, 15,
                          &mgp)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    return 0;
}

extern "C" int hsa_pass_times(hsa_index_t *ix, int n, float *widths_ms, float *search_ms)
{
    if (n < 1 || n > hsa_index::PASS_RING || (uint64_t)n > ix->pev_n) {
        hsa_set_error("hsa_pass_times: %d passes requested, %llu recorded (ring %d)", n,
                      (unsigned long long)ix->pev_n, hsa_index::PASS_RING);
        return HSA_E_ARG;
    }
    for (int i = 0; i < n; ++i) {
        hipEvent_t *pe = ix->pev[(ix->pev_n - (uint64_t)n + (uint64_t)i) % hsa_index::PASS_RING];
        HSA_HIP(hipEventSynchronize(pe[2]));
        HSA_HIP(hipEventElapsedTime(widths_ms + i, pe[0], pe[1]));
        HSA_HIP(hipEventElapsedTime(search_ms + i, pe[1], pe[2]));
    }
    return 0;
}

extern "C" int hsa_last_pass_ms(hsa_index_t *ix, float *widths_ms, float *search_ms)
{
    if (ix->pev_n) return hsa_pass_times(ix, 1, widths_ms, search_ms);   // the newest hsa_search_device pass
    HSA_HIP(hipEventSynchronize(ix->ev1));
    HSA_HIP(hipEventElapsedTime(widths_ms, ix->ev0, ix->evm));
    HSA_HIP(hipEventElapsedTime(search_ms, ix->evm, ix->ev1));
    return 0;
}
