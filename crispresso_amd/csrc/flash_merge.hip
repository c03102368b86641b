// Paired-end read merge on gfx950 with FLASH 1.2.11 semantics (include/crispr_flash.h).
//
// Replaces the FLASH process CRISPResso runs before the alignment
// (CRISPResso/CRISPRessoCORE.py:1655-1677); the algorithm is the one
// oracle/flash_oracle.py restates (Merger.align / combine / merge_pair).
//
// One wavefront per read pair.  The pair's read 1 and reverse-complemented read 2
// (bases canonicalised to A C G T N, qualities minus the offset, read 2's reversed)
// are staged in LDS; lane l scores the overlap positions l, l + 64, ... of the
// innie scan (read 2 under read 1 at position pos >= 0) and then of the outie scan
// (read 1 under read 2 at pos >= 1): mismatches and the sum of min(q1, q2) at the
// mismatches over min(overlap, max_overlap) bases, density = mismatches / that
// length in fp32 (the restatement's arithmetic, correctly rounded division).  The
// wave then takes the lexicographic minimum of (density, quality score, scan
// order) -- the restatement's "d < best or (d == best and q < best_q)" over the
// scan order -- and writes the merged read.  Integer / byte work plus two fp32
// divisions per position: VALU-bound, tens of bytes per pair.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crispr_flash.h"

namespace nwf {

constexpr int kMaxLen = 4096;
constexpr int kWpb = 4;

struct Args {
    const uint8_t* seq1;
    const uint8_t* qual1;
    const int64_t* off1;
    const uint8_t* seq2;
    const uint8_t* qual2;
    const int64_t* off2;
    int64_t n;
    uint8_t* out_seq;
    uint8_t* out_qual;
    int32_t* out_len;
    int32_t* out_flags;
    int32_t min_ov, max_ov, allow_outies, phred, cap;
    float max_density;
    int32_t lbuf;   // LDS bytes per staged read (>= longest read, 16-B multiple)
};

__device__ __forceinline__ uint8_t canon(uint8_t c) {
    const uint8_t u = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    return (u == 'A' || u == 'C' || u == 'G' || u == 'T') ? u : (uint8_t)'N';
}
__device__ __forceinline__ uint8_t comp(uint8_t c) {   // c in A C G T N
    return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'N';
}

// order-preserving unsigned image of an fp32 value (negatives below positives)
__device__ __forceinline__ unsigned ord32(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// best candidate so far: (density, quality score, scan order) as unsigned keys
struct Cand {
    unsigned d, q, o;
};
__device__ __forceinline__ bool better(const Cand& x, const Cand& y) {
    return x.d < y.d || (x.d == y.d && (x.q < y.q || (x.q == y.q && x.o < y.o)));
}

__global__ __launch_bounds__(64 * kWpb) void nwf_merge_kernel(const Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned char* r1 = smem + wave * 4 * a.lbuf;   // read 1 bases
    unsigned char* q1 = r1 + a.lbuf;                // read 1 qualities - offset (as int8 wraps)
    unsigned char* r2 = q1 + a.lbuf;                // read 2 reverse complement
    unsigned char* q2 = r2 + a.lbuf;                // read 2 qualities, reversed
    for (int64_t p = (int64_t)blockIdx.x * kWpb + wave; p < a.n; p += (int64_t)gridDim.x * kWpb) {
        const int64_t o1 = a.off1[p], o2 = a.off2[p];
        const int n1 = (int)(a.off1[p + 1] - o1), n2 = (int)(a.off2[p + 1] - o2);
        for (int k = lane; k < n1; k += 64) {
            r1[k] = canon(a.seq1[o1 + k]);
            q1[k] = (uint8_t)(a.qual1[o1 + k] - a.phred);
        }
        for (int k = lane; k < n2; k += 64) {
            r2[n2 - 1 - k] = comp(canon(a.seq2[o2 + k]));
            q2[n2 - 1 - k] = (uint8_t)(a.qual2[o2 + k] - a.phred);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        Cand best = {0xffffffffu, 0xffffffffu, 0xffffffffu};
        // one scan: b's start under a[pos], pos in [first, na - min_ov]
        auto scan = [&](const unsigned char* ra, const unsigned char* qa, int na, const unsigned char* rb,
                        const unsigned char* qb, int nb, int first, unsigned order0) {
            const int last = na - a.min_ov;
            if (last < first || nb < a.min_ov) return;
            for (int pos = first + lane; pos <= last; pos += 64) {
                const int eff = min(min(na - pos, nb), a.max_ov);
                // past lim mismatches the density exceeds max_density by more than 1/eff
                // (far above fp32 rounding): the overlap can never be taken, and when no
                // overlap can be, the pair stays uncombined whichever is "best" -- stop
                const int lim = (int)(a.max_density * (float)eff) + 1;
                int mm = 0, qt = 0;
                // 4 bases per step: b's dword is aligned, a's is assembled from two
                // aligned dwords (v_alignbyte); mismatching bytes = nonzero bytes of a ^ b
                const unsigned* a32 = (const unsigned*)ra;
                const unsigned* b32 = (const unsigned*)rb;
                const unsigned* qa32 = (const unsigned*)qa;
                const unsigned* qb32 = (const unsigned*)qb;
                auto mism = [&](int k, int ak) {   // mismatch flags (bit 7 of each byte) of bases k .. k+3
                    const unsigned x =
                        __builtin_amdgcn_alignbyte(a32[(ak >> 2) + 1], a32[ak >> 2], ak & 3) ^ b32[k >> 2];
                    unsigned m = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
                    const int rem = eff - k;
                    return rem < 4 ? m & ((1u << (8 * rem)) - 1u) : m;
                };
                // pass 1: mismatches only, abandoned past lim (most positions)
                for (int k = 0; k < eff && mm <= lim; k += 4) mm += __builtin_popcount(mism(k, pos + k));
                if (mm > lim) continue;
                // pass 2 (positions that can be taken): the qualities at the mismatches
                for (int k = 0; k < eff; k += 4) {
                    const int ak = pos + k;
                    unsigned m = mism(k, ak);
                    if (m) {
                        const unsigned qaw = __builtin_amdgcn_alignbyte(qa32[(ak >> 2) + 1], qa32[ak >> 2], ak & 3);
                        const unsigned qbw = qb32[k >> 2];
                        do {   // signed: quality - offset
                            const int b8 = (int)__builtin_ctz(m) - 7;   // 8 * byte index
                            qt += min((int)(signed char)(qaw >> b8), (int)(signed char)(qbw >> b8));
                            m &= m - 1u;
                        } while (m);
                    }
                }
                const float fe = (float)eff;
                const float d = (float)mm / fe, qs = (float)qt / fe;
                const Cand c = {ord32(d), ord32(qs), order0 + (unsigned)pos};
                if (better(c, best)) best = c;
            }
        };
        scan(r1, q1, n1, r2, q2, n2, 0, 0u);
        if (a.allow_outies) scan(r2, q2, n2, r1, q1, n1, 1, 1u << 20);
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const Cand o = {(unsigned)__shfl_xor((int)best.d, s), (unsigned)__shfl_xor((int)best.q, s),
                            (unsigned)__shfl_xor((int)best.o, s)};
            if (better(o, best)) best = o;
        }
        const int64_t ob = o1 + o2;
        const bool combined = best.o != 0xffffffffu && best.d <= ord32(a.max_density);
        if (!combined) {
            if (lane == 0) {
                a.out_len[p] = 0;
                a.out_flags[p] = 0;
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        const bool outie = best.o >= (1u << 20);
        const int pos = (int)(best.o & ((1u << 20) - 1));
        const unsigned char* ra = outie ? r2 : r1;
        const unsigned char* qa = outie ? q2 : q1;
        const unsigned char* rb = outie ? r1 : r2;
        const unsigned char* qb = outie ? q1 : q2;
        const int na = outie ? n2 : n1, nb = outie ? n1 : n2;
        const int ov = min(na - pos, nb);
        const int total = nb > ov ? pos + nb : na;
        for (int k = lane; k < total; k += 64) {
            uint8_t base, q;
            if (k < pos) {
                base = ra[k];
                q = qa[k];
            } else if (k < pos + ov) {
                const uint8_t sa = ra[k], sb = rb[k - pos];
                const int qa_k = (int)(signed char)qa[k], qb_k = (int)(signed char)qb[k - pos];
                if (sa == sb) {
                    base = sa;
                    q = (uint8_t)max(qa_k, qb_k);
                } else {
                    base = qa_k > qb_k ? sa : sb;
                    int mq = max(abs(qa_k - qb_k), 2);
                    if (a.cap) mq = min(mq, 2);
                    q = (uint8_t)mq;
                }
            } else if (nb > ov) {
                base = rb[k - pos];
                q = qb[k - pos];
            } else {
                base = ra[k];
                q = qa[k];
            }
            a.out_seq[ob + k] = base;
            a.out_qual[ob + k] = (uint8_t)(q + a.phred);
        }
        if (lane == 0) {
            a.out_len[p] = total;
            a.out_flags[p] = NWF_COMBINED | (outie ? NWF_OUTIE : 0);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace nwf

extern "C" const char* nwf_last_error(void) { return nwf::g_err.c_str(); }

extern "C" int nwf_merge_batch(int device, const nwf_params* params, const uint8_t* seq1, const uint8_t* qual1,
                               const int64_t* off1, const uint8_t* seq2, const uint8_t* qual2, const int64_t* off2,
                               int64_t n, uint8_t* out_seq, uint8_t* out_qual, int32_t* out_len, int32_t* out_flags,
                               float* kernel_ms) {
    using namespace nwf;
    if (!params || n < 0 || (n > 0 && (!off1 || !off2 || !out_len || !out_flags)))
        return fail(-1, "nwf_merge_batch: null argument or negative count");
    if (params->min_overlap < 1 || params->max_overlap < 1)
        return fail(-1, "nwf_merge_batch: min_overlap and max_overlap must be >= 1");
    if (kernel_ms) *kernel_ms = 0.0f;
    if (n == 0) return 0;
    const int64_t t1 = off1[n] - off1[0], t2 = off2[n] - off2[0];
    if (off1[0] != 0 || off2[0] != 0) return fail(-1, "nwf_merge_batch: offsets must start at 0");
    int lmax = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t l1 = off1[i + 1] - off1[i], l2 = off2[i + 1] - off2[i];
        if (l1 < 0 || l2 < 0) return fail(-1, "nwf_merge_batch: offsets not ascending");
        lmax = (int)std::max<int64_t>(lmax, std::max(l1, l2));
    }
    if (lmax > kMaxLen) return fail(-3, "nwf_merge_batch: reads longer than 4096 bases are not supported");
    if (hipSetDevice(device) != hipSuccess) return fail(-4, "nwf_merge_batch: hipSetDevice failed");
    std::vector<void*> bufs;
    auto dev = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        bufs.push_back(p);
        return p;
    };
    auto cleanup = [&]() {
        for (void* p : bufs) (void)hipFree(p);
    };
    Args a{};
    // + 8 bytes of slack after each buffer (none is read, but a reader never runs off an allocation)
    uint8_t* d_s1 = (uint8_t*)dev(t1 + 8);
    uint8_t* d_q1 = (uint8_t*)dev(t1 + 8);
    uint8_t* d_s2 = (uint8_t*)dev(t2 + 8);
    uint8_t* d_q2 = (uint8_t*)dev(t2 + 8);
    int64_t* d_o1 = (int64_t*)dev(sizeof(int64_t) * (n + 1));
    int64_t* d_o2 = (int64_t*)dev(sizeof(int64_t) * (n + 1));
    uint8_t* d_os = (uint8_t*)dev(t1 + t2 + 8);
    uint8_t* d_oq = (uint8_t*)dev(t1 + t2 + 8);
    int32_t* d_len = (int32_t*)dev(sizeof(int32_t) * n);
    int32_t* d_flg = (int32_t*)dev(sizeof(int32_t) * n);
    if (!d_s1 || !d_q1 || !d_s2 || !d_q2 || !d_o1 || !d_o2 || !d_os || !d_oq || !d_len || !d_flg) {
        cleanup();
        return fail(-4, "nwf_merge_batch: hipMalloc failed");
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool ok = hipMemcpy(d_s1, seq1, t1, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_q1, qual1, t1, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_s2, seq2, t2, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_q2, qual2, t2, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_o1, off1, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_o2, off2, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) == hipSuccess &&
              hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess;
    if (ok) {
        a.seq1 = d_s1;
        a.qual1 = d_q1;
        a.off1 = d_o1;
        a.seq2 = d_s2;
        a.qual2 = d_q2;
        a.off2 = d_o2;
        a.n = n;
        a.out_seq = d_os;
        a.out_qual = d_oq;
        a.out_len = d_len;
        a.out_flags = d_flg;
        a.min_ov = params->min_overlap;
        a.max_ov = params->max_overlap;
        a.allow_outies = params->allow_outies;
        a.phred = params->phred_offset;
        a.cap = params->cap_mismatch_quals;
        a.max_density = params->max_mismatch_density;
        a.lbuf = (lmax + 16 + 15) & ~15;
        const size_t lds = (size_t)4 * a.lbuf * kWpb;
        int dev_cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            dev_cus = prop.multiProcessorCount;
        const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n + kWpb - 1) / kWpb, (int64_t)dev_cus * 16));
        ok = hipEventRecord(e0, nullptr) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(nwf_merge_kernel, dim3((unsigned)grid), dim3(64 * kWpb), lds, nullptr, a);
            ok = hipGetLastError() == hipSuccess && hipEventRecord(e1, nullptr) == hipSuccess &&
                 hipEventSynchronize(e1) == hipSuccess;
        }
        if (ok && kernel_ms) ok = hipEventElapsedTime(kernel_ms, e0, e1) == hipSuccess;
        ok = ok && hipMemcpy(out_len, d_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(out_flags, d_flg, sizeof(int32_t) * n, hipMemcpyDeviceToHost) == hipSuccess &&
             (!out_seq || hipMemcpy(out_seq, d_os, t1 + t2, hipMemcpyDeviceToHost) == hipSuccess) &&
             (!out_qual || hipMemcpy(out_qual, d_oq, t1 + t2, hipMemcpyDeviceToHost) == hipSuccess);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    cleanup();
    if (!ok) return fail(-4, std::string("nwf_merge_batch: HIP error: ") + hipGetErrorString(hipGetLastError()));
    return 0;
}
