// gz_inflate.cpp -- parallel decompression of one gzip member (gz_inflate.h has the scheme).
//
// DEFLATE as RFC 1951 defines it: blocks of stored bytes, or of symbols in a fixed or a
// dynamic (header-described) canonical Huffman code; literal/length symbols 0..285,
// distance symbols 0..29, back-references of 3..258 bytes up to 32768 bytes back.  gzip
// framing as RFC 1952: a 10-byte header with optional extra / name / comment / header-CRC
// fields, the deflate stream, then CRC-32 and the size mod 2^32 of the data.
#include "gz_inflate.h"

#include <sys/mman.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "host_pool.h"

namespace nw_gz {

void Buffer::release() {
    if (p) munmap(p, cap);
    p = nullptr;
    n = cap = 0;
}

namespace {

// ------------------------------------------------------------------ fixed tables

struct Static {
    uint16_t len_base[29];
    uint8_t len_extra[29];
    uint16_t dist_base[30];
    uint8_t dist_extra[30];
    Static() {
        int b = 3;   // length symbols 257..284: groups of four per extra-bit count, 285 = 258
        for (int i = 0; i < 28; ++i) {
            const int e = i < 8 ? 0 : (i - 4) / 4;
            len_base[i] = (uint16_t)b;
            len_extra[i] = (uint8_t)e;
            b += 1 << e;
        }
        len_base[28] = 258;
        len_extra[28] = 0;
        b = 1;   // distance symbols: pairs per extra-bit count
        for (int i = 0; i < 30; ++i) {
            const int e = i < 4 ? 0 : (i - 2) / 2;
            dist_base[i] = (uint16_t)b;
            dist_extra[i] = (uint8_t)e;
            b += 1 << e;
        }
    }
};
const Static& S() {
    static const Static s;
    return s;
}

constexpr int kCodeOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ------------------------------------------------------------------ bit input

// LSB-first bits over a buffer padded with kPad readable bytes past the stream (a header
// read checks `over` once per code-length symbol: < 1 KiB past `lim`).  Invariant:
// bits [cnt, 64) of `buf` are zero or the stream's own next bits, so a refill may OR in
// whole words.
constexpr size_t kPad = 4096;

struct Bits {
    const uint8_t* base;
    const uint8_t* p;
    const uint8_t* lim;
    uint64_t buf = 0;
    unsigned cnt = 0;
    Bits(const uint8_t* b, const uint8_t* l, uint64_t bitpos) : base(b), p(b + (bitpos >> 3)), lim(l) {
        refill();
        const unsigned skip = (unsigned)(bitpos & 7);
        buf >>= skip;
        cnt -= skip;
    }
    void refill() {
        uint64_t w;
        std::memcpy(&w, p, 8);
        buf |= w << cnt;
        p += (63 - cnt) >> 3;
        cnt |= 56;
    }
    bool over() const { return p > lim; }
    uint64_t pos() const { return (uint64_t)(p - base) * 8 - cnt; }
    uint32_t peek(unsigned n) const { return (uint32_t)(buf & ((1ull << n) - 1)); }
    void drop(unsigned n) {
        buf >>= n;
        cnt -= n;
    }
    uint32_t get(unsigned n) {   // n <= 32
        if (cnt < n) refill();
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
};

// ------------------------------------------------------------------ Huffman tables

// entry: bits 0..15 symbol (or subtable offset), 16..19 code length (0: no code here),
// bit 20: subtable pointer.  Codes longer than `pb` bits continue in a subtable of
// 2^(15 - pb) entries indexed by the next bits.
struct Table {
    int pb = 0;
    std::vector<uint32_t> e;
    enum Kind { kCodes, kLens, kDists };
    // false: over-subscribed, or incomplete where RFC 1951 decoders (zlib) refuse it
    bool build(const uint8_t* len, int n, int bits, Kind kind) {
        pb = bits;
        int count[16] = {0};
        for (int s = 0; s < n; ++s) count[len[s]]++;
        count[0] = 0;
        int left = 1, maxl = 0;
        for (int l = 1; l <= 15; ++l) {
            left = (left << 1) - count[l];
            if (left < 0) return false;
            if (count[l]) maxl = l;
        }
        if (left > 0 && maxl != 0 && (kind == kCodes || maxl != 1)) return false;
        if (maxl == 0 && kind != kDists) return false;
        const int psize = 1 << pb, ssize = 1 << (15 - pb);
        int nsub = 0;
        e.assign((size_t)psize, 0);
        int next[16];
        int code = 0;
        for (int l = 1; l <= 15; ++l) {
            code = (code + count[l - 1]) << 1;
            next[l] = code;
        }
        for (int s = 0; s < n; ++s) {
            const int l = len[s];
            if (!l) continue;
            const int c = next[l]++;
            int r = 0;   // the code's bits in stream order
            for (int k = 0; k < l; ++k) r |= ((c >> k) & 1) << (l - 1 - k);
            const uint32_t ent = (uint32_t)s | (uint32_t)l << 16;
            if (l <= pb) {
                for (int i = r; i < psize; i += 1 << l) e[(size_t)i] = ent;
            } else {
                const int pi = r & (psize - 1);
                if (!(e[(size_t)pi] & (1u << 20))) {
                    const size_t off = (size_t)psize + (size_t)nsub++ * (size_t)ssize;
                    e.resize(off + (size_t)ssize, 0);
                    e[(size_t)pi] = (uint32_t)off | (uint32_t)pb << 16 | 1u << 20;
                }
                const size_t off = e[(size_t)pi] & 0xFFFF;
                for (int i = r >> pb; i < ssize; i += 1 << (l - pb)) e[off + (size_t)i] = ent;
            }
        }
        return true;
    }
    // the next symbol, or -1 (no code); needs >= 15 bits in b
    int decode(Bits& b) const {
        uint32_t x = e[b.peek((unsigned)pb)];
        if (x & (1u << 20)) x = e[(x & 0xFFFF) + ((b.buf >> pb) & ((1u << (15 - pb)) - 1))];
        const unsigned l = (x >> 16) & 15;
        if (!l) return -1;
        b.drop(l);
        return (int)(x & 0xFFFF);
    }
};

struct Fixed {
    Table L, D;
    Fixed() {
        uint8_t l[288], d[30];
        for (int i = 0; i < 288; ++i) l[i] = (uint8_t)(i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8);
        for (int i = 0; i < 30; ++i) d[i] = 5;
        L.build(l, 288, 10, Table::kLens);
        D.build(d, 30, 8, Table::kDists);
    }
};
const Fixed& fixed_tables() {
    static const Fixed f;
    return f;
}

// A dynamic block's header (after BFINAL / BTYPE) into L / D; false: not a valid header.
bool read_dynamic(Bits& b, Table& L, Table& D) {
    const int hlit = (int)b.get(5) + 257, hdist = (int)b.get(5) + 1, hclen = (int)b.get(4) + 4;
    if (hlit > 286 || hdist > 30) return false;
    uint8_t cl[19] = {0};
    for (int i = 0; i < hclen; ++i) cl[kCodeOrder[i]] = (uint8_t)b.get(3);
    Table C;
    if (!C.build(cl, 19, 7, Table::kCodes)) return false;
    uint8_t lens[320];
    int i = 0;
    const int tot = hlit + hdist;
    while (i < tot) {
        if (b.over()) return false;
        if (b.cnt < 32) b.refill();
        const int sym = C.decode(b);
        if (sym < 0) return false;
        if (sym < 16) {
            lens[i++] = (uint8_t)sym;
            continue;
        }
        int rep;
        uint8_t val = 0;
        if (sym == 16) {
            if (i == 0) return false;
            val = lens[i - 1];
            rep = 3 + (int)b.get(2);
        } else if (sym == 17) {
            rep = 3 + (int)b.get(3);
        } else {
            rep = 11 + (int)b.get(7);
        }
        if (i + rep > tot) return false;
        std::memset(lens + i, val, (size_t)rep);
        i += rep;
    }
    if (lens[256] == 0) return false;
    return L.build(lens, hlit, 10, Table::kLens) && D.build(lens + hlit, hdist, 8, Table::kDists);
}

// ------------------------------------------------------------------ output sinks

// Output positions are indices into a sink's array `p`; the kWin entries before a range's
// first byte hold the 32 KiB before it (markers 256 + i in the first pass, the bytes in the
// second), so a back-reference reads p[n - dist] without a branch.  room(): called when
// fewer than kRoom entries are left before `cap`; it makes room (slides, or moves to the
// next buffer) or fails.  Copies may write up to 16 entries past a match's end.
constexpr size_t kWin = 32768;
constexpr size_t kRoom = 258 + 16;

// First pass: 16-bit symbols in a cache-sized sliding buffer; only the count and the last
// 32 KiB are kept.
struct Ring16 {
    static constexpr size_t kLen = kWin + ((size_t)1 << 19);
    std::vector<uint16_t> buf;
    uint16_t* p;
    size_t n = kWin, cap = kLen;
    size_t slid = 0;   // symbols moved out of the buffer's front
    Ring16() : buf(kLen + 64) {
        p = buf.data();
        for (size_t i = 0; i < kWin; ++i) p[i] = (uint16_t)(256 + i);
    }
    void reset() {
        for (size_t i = 0; i < kWin; ++i) p[i] = (uint16_t)(256 + i);
        n = kWin;
        slid = 0;
    }
    bool room() {
        std::memmove(p, p + n - kWin, kWin * sizeof(uint16_t));
        slid += n - kWin;
        n = kWin;
        return true;
    }
    size_t produced() const { return slid + n - kWin; }
};

// Second pass: bytes straight into the range's place in the output [dst, dst + m) (m known
// from the first pass).  The first 32 KiB are decoded in a staging buffer behind the window
// (references before the range's start read the window, not the previous range's bytes,
// which another thread is writing), the middle in place, and the last kRoom bytes in a
// staging buffer again (the copies' overrun must not reach the next range).
struct Bytes8 {
    unsigned char* dst;
    size_t m;
    std::vector<unsigned char> stage;
    unsigned char* p;
    size_t n = kWin, cap;
    int mode = 0;   // 0 head (stage), 1 body (in place), 2 tail (stage)
    size_t tail_at = 0;   // range offset of the tail stage's first byte
    Bytes8(unsigned char* d, size_t m_, const unsigned char* window) : dst(d), m(m_), stage(3 * kWin + 64) {
        p = stage.data();
        std::memcpy(p, window, kWin);
        cap = 3 * kWin;
    }
    bool room() {
        if (mode == 0) {
            const size_t got = n - kWin;
            if (got + kRoom + kWin > m) return to_tail(got);   // a short range: straight to the tail
            std::memcpy(dst, p + kWin, got);
            p = dst - kWin;   // p[n] is dst[n - kWin]; p[n - dist] >= dst once got >= kWin
            cap = kWin + m;
            mode = 1;
            return n + kRoom <= cap || to_tail(got);
        }
        if (mode == 1) return to_tail(n - kWin);
        return false;   // more than m bytes: not the first pass's stream
    }
    bool to_tail(size_t got) {
        // the stage holds the 32 KiB before range offset `got`, then the rest of the range
        unsigned char* s = stage.data();
        if (mode == 0) {
            std::memmove(s, p + got, kWin);   // (got < kWin + kRoom: the window and what followed)
            std::memcpy(dst, p + kWin, got);
        } else {
            std::memcpy(s, dst + got - kWin, kWin);
        }
        p = s;
        n = kWin;
        cap = 3 * kWin;
        tail_at = got;
        mode = 2;
        return m - got + kRoom <= 2 * kWin;   // the rest fits the stage
    }
    bool finish() {
        if (mode == 0) {
            if (n - kWin != m) return false;
            std::memcpy(dst, p + kWin, m);
            return true;
        }
        if (mode == 1) return n - kWin == m;
        if (tail_at + (n - kWin) != m) return false;
        std::memcpy(dst + tail_at, p + kWin, n - kWin);
        return true;
    }
};

enum { kOk = 0, kEnd = 1, kBad = -1 };

inline bool text_byte(int c) { return c == '\n' || c == '\r' || c == '\t' || (c >= 32 && c < 127); }

template <class T>
inline void copy_match(T* dst, size_t dist, size_t len) {
    const T* src = dst - dist;
    constexpr size_t kStep = 16 / sizeof(T);
    if (dist >= kStep) {
        for (size_t k = 0; k < len; k += kStep) std::memcpy(dst + k, src + k, 16);
    } else if (dist == 1) {
        std::fill_n(dst, len, *src);
    } else {
        for (size_t k = 0; k < len; ++k) dst[k] = src[k];
    }
}

// The symbols of one block up to its end-of-block code.  `text`: only text bytes may be
// literals (the candidate check: FASTQ is text).
template <class Sink>
int decode_block(Bits& b, const Table& L, const Table& D, Sink& o, bool text) {
    const Static& st = S();
    for (;;) {
        if (o.n + kRoom > o.cap && !o.room()) return kBad;
        if (b.over()) return kBad;
        if (b.cnt < 48) b.refill();
        int sym = L.decode(b);
        if (sym < 256) {
            if (sym < 0 || (text && !text_byte(sym))) return kBad;
            o.p[o.n++] = (decltype(o.p[0] + 0))sym;
            // a second literal without a refill when the bits are there
            const uint32_t x0 = L.e[b.peek((unsigned)L.pb)];
            if (!(x0 & (1u << 20)) && ((x0 >> 16) & 15) && (x0 & 0xFFFF) < 256 && b.cnt >= ((x0 >> 16) & 15)) {
                const int s2 = (int)(x0 & 0xFFFF);
                if (text && !text_byte(s2)) return kBad;
                b.drop((x0 >> 16) & 15);
                o.p[o.n++] = (decltype(o.p[0] + 0))s2;
            }
            continue;
        }
        if (sym == 256) return kEnd;
        sym -= 257;
        if (sym >= 29) return kBad;
        const unsigned le = st.len_extra[sym];
        const size_t len = st.len_base[sym] + (le ? b.get(le) : 0);
        if (b.cnt < 32) b.refill();
        const int ds = D.decode(b);
        if (ds < 0 || ds >= 30) return kBad;
        const unsigned de = st.dist_extra[ds];
        const size_t dist = st.dist_base[ds] + (de ? b.get(de) : 0);
        copy_match(o.p + o.n, dist, len);
        o.n += len;
    }
}

// Blocks from the bit position in b until the block boundary `stop` (a bit position;
// UINT64_MAX: the final block).  kOk: ended exactly there (or after the final block, *end
// = the bit position after it); kBad: a bad block, a final block before `stop`, or a
// boundary past `stop` without one at it.
template <class Sink>
int decode_range(Bits& b, Sink& o, uint64_t stop, uint64_t* end) {
    const Fixed& F = fixed_tables();
    Table L, D;
    for (;;) {
        const uint64_t at = b.pos();
        if (stop != UINT64_MAX) {
            if (at == stop) return kOk;
            if (at > stop) return kBad;
        }
        if (b.over()) return kBad;
        if (b.cnt < 32) b.refill();
        const uint32_t hdr = b.get(3);
        const bool final = hdr & 1;
        const uint32_t type = hdr >> 1;
        int r;
        if (type == 0) {   // stored: byte-aligned LEN, ~LEN, bytes
            b.drop(b.cnt & 7);
            const uint64_t bytepos = b.pos() >> 3;
            const uint8_t* q = b.base + bytepos;
            if (q + 4 > b.lim) return kBad;
            const uint32_t len = (uint32_t)q[0] | (uint32_t)q[1] << 8, nlen = (uint32_t)q[2] | (uint32_t)q[3] << 8;
            if ((len ^ 0xFFFF) != nlen || q + 4 + len > b.lim) return kBad;
            for (uint32_t k = 0; k < len;) {
                if (o.n + kRoom > o.cap && !o.room()) return kBad;
                const uint32_t piece = std::min<uint32_t>(len - k, 256);
                for (uint32_t j = 0; j < piece; ++j) o.p[o.n + j] = q[4 + k + j];
                o.n += piece;
                k += piece;
            }
            b = Bits(b.base, b.lim, (bytepos + 4 + len) * 8);
            r = kEnd;
        } else if (type == 1) {
            r = decode_block(b, F.L, F.D, o, false);
        } else if (type == 2) {
            if (!read_dynamic(b, L, D)) return kBad;
            r = decode_block(b, L, D, o, false);
        } else {
            return kBad;
        }
        if (r != kEnd) return kBad;
        if (final) {
            if (stop != UINT64_MAX) return kBad;
            *end = b.pos();
            return kOk;
        }
    }
}

// the candidate check's sink: a bounded Ring16 (a block of more than 16M symbols is not
// taken as a candidate)
struct Probe16 : Ring16 {
    bool room() {
        if (produced() > ((size_t)16 << 20)) return false;
        return Ring16::room();
    }
};

// The first bit position in [lo, hi) where a dynamic block (not final) starts whose header
// is valid and whose symbols decode to text up to its end, followed by a block header that
// is not reserved.  UINT64_MAX: none.
uint64_t find_block(const uint8_t* base, const uint8_t* lim, uint64_t lo, uint64_t hi) {
    Table L, D;
    Probe16 scratch;
    for (uint64_t at = lo; at < hi; ++at) {
        const uint8_t* q = base + (at >> 3);
        uint32_t w;
        std::memcpy(&w, q, 4);
        w >>= (at & 7);
        // BFINAL 0, BTYPE 2 (bits 0b100), HLIT <= 29, HDIST <= 29
        if ((w & 7) != 4 || ((w >> 3) & 31) > 29 || ((w >> 8) & 31) > 29) continue;
        Bits b(base, lim, at + 3);
        if (!read_dynamic(b, L, D)) continue;
        scratch.reset();
        if (decode_block(b, L, D, scratch, true) != kEnd) continue;
        if (b.over()) continue;
        if (b.cnt < 8) b.refill();
        if (((b.buf >> 1) & 3) == 3) continue;
        return at;
    }
    return UINT64_MAX;
}

// gzip header length; 0: not a gzip member this reader takes
size_t gzip_header(const uint8_t* p, size_t n) {
    if (n < 18 || p[0] != 0x1f || p[1] != 0x8b || p[2] != 8) return 0;
    const uint8_t flg = p[3];
    if (flg & 0xE0) return 0;
    size_t at = 10;
    if (flg & 4) {   // FEXTRA
        if (at + 2 > n) return 0;
        at += 2 + ((size_t)p[at] | (size_t)p[at + 1] << 8);
    }
    for (int f : {8, 16}) {   // FNAME, FCOMMENT: zero-terminated
        if (!(flg & f)) continue;
        while (at < n && p[at]) ++at;
        ++at;
    }
    if (flg & 2) at += 2;   // FHCRC
    return at + 8 <= n ? at : 0;
}

}  // namespace

bool inflate_parallel(const unsigned char* file, size_t n, int threads, Crc32Fn crc, Buffer* out) {
    *out = Buffer{};
    const size_t hdr = gzip_header(file, n);
    if (!hdr || threads < 2 || n < ((size_t)4 << 20)) return false;
    const size_t isize = (size_t)file[n - 4] | (size_t)file[n - 3] << 8 | (size_t)file[n - 2] << 16 |
                         (size_t)file[n - 1] << 24;
    const uint32_t want_crc = (uint32_t)file[n - 8] | (uint32_t)file[n - 7] << 8 | (uint32_t)file[n - 6] << 16 |
                              (uint32_t)file[n - 5] << 24;
    // the deflate bytes, padded (the bit reader reads whole words)
    const size_t dn = n - 8 - hdr;
    std::vector<uint8_t> data(dn + kPad, 0);
    std::memcpy(data.data(), file + hdr, dn);
    const uint8_t* base = data.data();
    const uint8_t* lim = base + dn + 8;   // bytes past the stream: the reader is lost

    nw_host::Pool& pool = nw_host::Pool::get();
    const int P = std::min(threads, pool.threads());
    if (P < 2) return false;
    // candidates: range k of the compressed bits starts its search at k * dn / P
    std::vector<uint64_t> cand((size_t)P, UINT64_MAX);
    cand[0] = 0;
    pool.run(P, [&](int k) {
        if (k == 0) return;
        int64_t lo, hi;
        nw_host::Pool::range((int64_t)dn, P, k, &lo, &hi);
        cand[(size_t)k] = find_block(base, lim, (uint64_t)lo * 8, (uint64_t)hi * 8);
    });
    std::vector<uint64_t> starts;
    for (uint64_t c : cand)
        if (c != UINT64_MAX) starts.push_back(c);
    const int C = (int)starts.size();
    if (C < 2) return false;
    // first pass: every range to the next range's start, 16-bit symbols, keeping its length
    // and its last 32 KiB
    std::vector<size_t> len((size_t)C, 0);
    std::vector<std::vector<uint16_t>> last((size_t)C);
    std::vector<int> rc((size_t)C, kBad);
    std::vector<uint64_t> end_bits((size_t)C, 0);
    pool.run(C, [&](int k) {
        const uint64_t stop = k + 1 < C ? starts[(size_t)k + 1] : UINT64_MAX;
        Ring16 o;
        Bits b(base, lim, starts[(size_t)k]);
        rc[(size_t)k] = decode_range(b, o, stop, &end_bits[(size_t)k]);
        len[(size_t)k] = o.produced();
        last[(size_t)k].assign(o.p + o.n - kWin, o.p + o.n);
    });
    for (int r : rc)
        if (r != kOk) return false;
    // one member, nothing after it: the stream ends in the byte before the trailer
    if ((end_bits[(size_t)C - 1] + 7) / 8 != dn) return false;
    std::vector<size_t> off((size_t)C + 1, 0);
    for (int k = 0; k < C; ++k) off[(size_t)k + 1] = off[(size_t)k] + len[(size_t)k];
    const size_t total = off[(size_t)C];
    if ((total & 0xFFFFFFFFu) != isize) return false;
    // the 32 KiB before each range, range by range (`known`: how many lie inside the stream)
    std::vector<std::vector<uint8_t>> window((size_t)C, std::vector<uint8_t>(kWin, 0));
    size_t known = 0;
    for (int k = 0; k + 1 < C; ++k) {
        const std::vector<uint8_t>& w = window[(size_t)k];
        std::vector<uint8_t>& nx = window[(size_t)k + 1];
        for (size_t i = 0; i < kWin; ++i) {
            const uint16_t v = last[(size_t)k][i];
            if (v >= 256 && (size_t)(v - 256) < kWin - known) return false;   // before the stream's start
            nx[i] = v < 256 ? (uint8_t)v : w[v - 256];
        }
        known = std::min(kWin, known + len[(size_t)k]);
    }
    // second pass: the bytes in place, and each range's CRC-32
    Buffer buf;
    buf.cap = total + 4096;
    void* m = mmap(nullptr, buf.cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) return false;
    (void)madvise(m, buf.cap, MADV_HUGEPAGE);
    buf.p = (unsigned char*)m;
    buf.n = total;
    std::vector<uint32_t> crcs((size_t)C, 0);
    std::vector<char> ok2((size_t)C, 0);
    pool.run(C, [&](int k) {
        Bytes8 o(buf.p + off[(size_t)k], len[(size_t)k], window[(size_t)k].data());
        Bits b(base, lim, starts[(size_t)k]);
        const uint64_t stop = k + 1 < C ? starts[(size_t)k + 1] : UINT64_MAX;
        uint64_t e = 0;
        if (decode_range(b, o, stop, &e) != kOk || !o.finish()) return;
        const unsigned char* d = buf.p + off[(size_t)k];
        // zlib's crc32 takes a 32-bit length: a range over 4 GiB (few block starts found in a
        // large member) goes through crc32_z's size_t length instead of being truncated
        crcs[(size_t)k] = crc ? crc(0, d, len[(size_t)k]) : (uint32_t)crc32_z(0, d, (z_size_t)len[(size_t)k]);
        ok2[(size_t)k] = 1;
    });
    uint32_t all = crcs[0];
    for (int k = 1; k < C; ++k) all = (uint32_t)crc32_combine(all, crcs[(size_t)k], (z_off_t)len[(size_t)k]);
    bool ok = all == want_crc;
    for (char g : ok2) ok &= g != 0;
    if (!ok) {
        buf.release();
        return false;
    }
    *out = buf;
    return true;
}

}  // namespace nw_gz
