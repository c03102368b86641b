// nw_pack.cpp -- host packer for nw_align_ops_packed (include/crispr_nw.h).
//
// 2 bits per base, A C T G = 0 1 2 3 = (byte >> 1) & 3 for A C G T a c g t; base at
// batch position i lives in bits 2 (i % 4) of byte i / 4.  Every other byte (N, IUPAC
// codes, U, '-', ...) is an exception: its position and the byte itself, in ascending
// position order.  Threads take byte ranges of the packed stream; a thread's
// exceptions are kept apart and joined in order.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/crispr_nw.h"
#include "host_pool.h"

namespace {

inline bool is_acgt(unsigned char b) {
    const unsigned char u = b & 0xDF;
    return u == 'A' || u == 'C' || u == 'G' || u == 'T';
}

// packed bytes [q0, q1) (bases 4 q0 .. 4 q1), batch bases [b0, b1) only
void pack_range(const unsigned char* reads, int64_t b0, int64_t b1, int64_t q0, int64_t q1, uint8_t* packed,
                std::vector<std::pair<int64_t, uint8_t>>* exc) {
    auto slow = [&](int64_t q) {
        unsigned v = 0;
        for (int k = 0; k < 4; ++k) {
            const int64_t i = 4 * q + k;
            if (i < b0 || i >= b1) continue;
            const unsigned char b = reads[i];
            if (is_acgt(b)) v |= (unsigned)((b >> 1) & 3) << (2 * k);
            else exc->emplace_back(i, b);
        }
        packed[q] = (uint8_t)v;
    };
    int64_t q = q0;
    for (; q < q1 && 4 * q < b0; ++q) slow(q);
    const int64_t qe = std::max(q, std::min(q1, b1 / 4));   // bytes whose 4 bases are all inside the batch
    // 16 bases per step: a vectorisable exception test, then the packing
    for (; q + 4 <= qe; q += 4) {
        const unsigned char* p = reads + 4 * q;
        unsigned bad = 0;
        for (int k = 0; k < 16; ++k) bad |= !is_acgt(p[k]);
        if (bad) {
            for (int t = 0; t < 4; ++t) slow(q + t);
            continue;
        }
        for (int t = 0; t < 4; ++t)
            packed[q + t] = (uint8_t)(((p[4 * t] >> 1) & 3) | (((p[4 * t + 1] >> 1) & 3) << 2) |
                                      (((p[4 * t + 2] >> 1) & 3) << 4) | (((p[4 * t + 3] >> 1) & 3) << 6));
    }
    for (; q < q1; ++q) slow(q);
}

}  // namespace

extern "C" int nw_pack_reads(const char* reads, const int64_t* offsets, int64_t n, uint8_t* packed, int64_t* exc_pos,
                             uint8_t* exc_byte, int64_t exc_cap, int64_t* n_exc, int32_t nthreads) {
    if (n < 0 || !offsets || !n_exc || (n > 0 && (!reads || !packed))) return NW_E_INVALID;
    *n_exc = 0;
    if (n == 0) return NW_OK;
    const int64_t b0 = offsets[0], b1 = offsets[n];
    if (b1 < b0) return NW_E_INVALID;
    const int64_t q0 = b0 / 4, q1 = (b1 + 3) / 4;
    int nt = nthreads > 0 ? nthreads : nw_host::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (q1 - q0) / (1 << 16) + 1));
    std::vector<std::vector<std::pair<int64_t, uint8_t>>> exc((size_t)nt);
    const int64_t per = ((q1 - q0 + nt - 1) / nt + 3) & ~(int64_t)3;
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) {
        const int64_t lo = q0 + t * per, hi = std::min(q1, lo + per);
        if (lo >= hi) continue;
        if (nt == 1) pack_range((const unsigned char*)reads, b0, b1, lo, hi, packed, &exc[(size_t)t]);
        else pool.emplace_back(pack_range, (const unsigned char*)reads, b0, b1, lo, hi, packed, &exc[(size_t)t]);
    }
    for (auto& th : pool) th.join();
    int64_t total = 0;
    for (auto& e : exc) total += (int64_t)e.size();
    *n_exc = total;
    if (total > exc_cap) return NW_E_CAPACITY;
    int64_t k = 0;
    for (auto& e : exc)
        for (auto& pr : e) {
            exc_pos[k] = pr.first;
            exc_byte[k] = pr.second;
            ++k;
        }
    return NW_OK;
}

// uint16 read lengths for nw_align_ops_packed_lens: one pass over the offsets on the host
// pool (nthreads <= 0: all of its threads; > 0: at most that many parts), contiguous ranges;
// NW_E_UNSUPPORTED when a length does not fit (or is negative).
extern "C" int nw_read_lengths16(const int64_t* offsets, int64_t n, uint16_t* lens, int32_t nthreads) {
    if (n < 0 || (n > 0 && (!offsets || !lens))) return NW_E_INVALID;
    nw_host::Pool& pool = nw_host::Pool::get();
    int nt = nthreads > 0 ? std::min(nthreads, pool.threads()) : pool.threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n >> 16));
    std::vector<char> bad((size_t)nt, 0);
    pool.run(nt, [&](int t) {
        int64_t lo, hi;
        nw_host::Pool::range(n, nt, t, &lo, &hi);
        bool b = false;
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t l = offsets[r + 1] - offsets[r];
            b |= (uint64_t)l > 65535u;
            lens[r] = (uint16_t)l;
        }
        bad[(size_t)t] = b;
    });
    for (char b : bad)
        if (b) return NW_E_UNSUPPORTED;
    return NW_OK;
}
