// nw_synth.cpp -- native generator of the synthetic read sets of SURVEY.md 8(d)
// (include/crispr_synth.h).  Bench / test input only: nothing on the aligner path
// calls it.
//
// Same mutation mix as crispresso_amd/synth.py (C2 / C4: 60 % exact copies, 20 % 1-3
// substitutions at uniform positions, 10 % one deletion of Geom(0.3) length truncated
// to 1-30 starting at La/2 +- 10, 5 % one insertion of 1-10 random bases at La/2 +- 10,
// 5 % 1 %-per-base substitution noise), but a counter-based RNG: every draw is
// splitmix64(seed, read, draw), so any read range is generated independently (threads,
// and a rank's 12.5M-read calls of C4 each generated on its own) and the lengths pass
// and the bytes pass agree without storing the draws.  synth.py takes ~3 s per 1M
// reads on the GPU box's host; this takes ~0.1 s on 16 threads.
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/crispr_synth.h"
#include "host_pool.h"

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// draw k of read r: 64 uniform bits
struct Rng {
    uint64_t base;
    uint64_t operator()(uint64_t k) const { return mix64(base ^ mix64(k)); }
    double unit(uint64_t k) const { return (double)((*this)(k) >> 11) * (1.0 / 9007199254740992.0); }
    int below(uint64_t k, int m) const { return (int)(((*this)(k) >> 32) * (uint64_t)m >> 32); }
};

constexpr char kBases[4] = {'A', 'C', 'G', 'T'};
enum Kind { EXACT = 0, SUBS, DEL, INS, NOISE };

// what a read is: its kind, the event position / size, its length
struct Plan {
    int kind, pos, size, len;
};

Plan plan_of(const Rng& g, int La, const double* cum) {
    Plan p{EXACT, 0, 0, La};
    const double u = g.unit(0);
    p.kind = u < cum[0] ? EXACT : u < cum[1] ? SUBS : u < cum[2] ? DEL : u < cum[3] ? INS : NOISE;
    const int centre = La / 2;
    auto clip = [&](int x) { return x < 1 ? 1 : (x > La - 1 ? La - 1 : x); };
    if (p.kind == DEL) {
        // Geom(0.3) on 1, 2, ...: 1 + floor(log U / log 0.7), truncated to 30
        const double v = 1.0 - g.unit(1);   // (0, 1]
        int d = 1 + (int)std::floor(std::log(v) / std::log(0.7));
        d = d > 30 ? 30 : d;
        p.pos = clip(centre + g.below(2, 21) - 10);
        if (d > La - p.pos - 1) d = La - p.pos - 1;
        p.size = d > 0 ? d : 0;
        p.len = La - p.size;
    } else if (p.kind == INS) {
        p.size = 1 + g.below(1, 10);
        p.pos = clip(centre + g.below(2, 21) - 10);
        p.len = La + p.size;
    } else if (p.kind == SUBS) {
        p.size = 1 + g.below(1, 3);
    }
    if (La <= 1) {   // nothing to mutate around
        p.kind = EXACT;
        p.len = La;
    }
    return p;
}

// a base different from b (uniform among the other three)
inline char other(char b, int r3) {
    int c = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3;
    return kBases[(c + 1 + r3) & 3];
}

void emit(const Rng& g, const char* amp, int La, const Plan& p, char* out) {
    switch (p.kind) {
        case EXACT:
            std::memcpy(out, amp, (size_t)La);
            break;
        case SUBS:
            std::memcpy(out, amp, (size_t)La);
            for (int k = 0; k < p.size; ++k) {
                const int at = g.below(10 + 2 * k, La);
                out[at] = other(out[at], g.below(11 + 2 * k, 3));
            }
            break;
        case DEL:
            std::memcpy(out, amp, (size_t)p.pos);
            std::memcpy(out + p.pos, amp + p.pos + p.size, (size_t)(La - p.pos - p.size));
            break;
        case INS:
            std::memcpy(out, amp, (size_t)p.pos);
            for (int k = 0; k < p.size; ++k) out[p.pos + k] = kBases[g.below(10 + k, 4)];
            std::memcpy(out + p.pos + p.size, amp + p.pos, (size_t)(La - p.pos));
            break;
        default:   // NOISE: every base substituted with probability 1 %
            for (int i = 0; i < La; ++i) {
                const uint64_t v = g(100 + (uint64_t)i);
                out[i] = (v & 0xffffffffull) < 42949673ull ? other(amp[i], (int)((v >> 32) % 3)) : amp[i];
            }
            break;
    }
}

bool cum_of(const double* mix, double* cum) {
    double t = 0.0;
    for (int k = 0; k < 5; ++k) {
        if (!(mix[k] >= 0.0)) return false;
        t += mix[k];
    }
    if (!(t > 0.0)) return false;
    double s = 0.0;
    for (int k = 0; k < 5; ++k) cum[k] = (s += mix[k] / t);
    return true;
}

inline Rng rng_of(uint64_t seed, int64_t r) { return Rng{mix64(seed * 0x632be59bd9b4e019ull + 0x1234567ull) ^ (uint64_t)r * 0xd1b54a32d192ed03ull}; }

}  // namespace

extern "C" {

int64_t nw_synth_offsets(const char* amp, int32_t La, int64_t first, int64_t n, uint64_t seed, const double* mix,
                         int64_t* offsets, int32_t nthreads) {
    double cum[5];
    if (!amp || La <= 0 || n < 0 || first < 0 || !offsets || !mix || !cum_of(mix, cum)) return -1;
    nw_host::Pool& pool = nw_host::Pool::get();
    const int parts = (int)std::min<int64_t>(std::min(nthreads > 0 ? nthreads : pool.threads(), pool.threads()),
                                             std::max<int64_t>(1, n >> 14));
    std::vector<int64_t> sums((size_t)parts + 1, 0);
    pool.run(parts, [&](int q) {
        int64_t lo, hi, s = 0;
        nw_host::Pool::range(n, parts, q, &lo, &hi);
        for (int64_t r = lo; r < hi; ++r) {
            s += plan_of(rng_of(seed, first + r), La, cum).len;
            offsets[r + 1] = s;   // part-relative for now
        }
        sums[(size_t)q + 1] = s;
    });
    for (int q = 0; q < parts; ++q) sums[(size_t)q + 1] += sums[(size_t)q];
    offsets[0] = 0;
    pool.run(parts, [&](int q) {
        int64_t lo, hi;
        nw_host::Pool::range(n, parts, q, &lo, &hi);
        for (int64_t r = lo; r < hi; ++r) offsets[r + 1] += sums[(size_t)q];
    });
    return offsets[n];
}

int nw_synth_reads(const char* amp, int32_t La, int64_t first, int64_t n, uint64_t seed, const double* mix,
                   const int64_t* offsets, char* buf, int32_t nthreads) {
    double cum[5];
    if (!amp || La <= 0 || n < 0 || first < 0 || !offsets || !buf || !mix || !cum_of(mix, cum)) return -1;
    nw_host::Pool& pool = nw_host::Pool::get();
    const int parts = (int)std::min<int64_t>(std::min(nthreads > 0 ? nthreads : pool.threads(), pool.threads()),
                                             std::max<int64_t>(1, n >> 14));
    std::vector<int> bad((size_t)parts, 0);
    pool.run(parts, [&](int q) {
        int64_t lo, hi;
        nw_host::Pool::range(n, parts, q, &lo, &hi);
        for (int64_t r = lo; r < hi; ++r) {
            const Rng g = rng_of(seed, first + r);
            const Plan p = plan_of(g, La, cum);
            if (offsets[r + 1] - offsets[r] != p.len) {
                bad[(size_t)q] = 1;
                return;
            }
            emit(g, amp, La, p, buf + (offsets[r] - offsets[0]));
        }
    });
    for (int b : bad)
        if (b) return -1;
    return 0;
}

}  // extern "C"
