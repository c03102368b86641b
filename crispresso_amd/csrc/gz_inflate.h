// gz_inflate.h -- parallel decompression of one gzip member (the FASTQ.gz ingest, nw_fastq.cpp).
//
// A gzip member is one DEFLATE stream (RFC 1951): blocks that start at arbitrary bit
// offsets, whose back-references reach up to 32 KiB into the output before them.  One
// thread decodes it at ~1.7 GB/s (libdeflate), which was most of the 1M-read ingest.  Here
// the compressed bytes are cut into one range per thread; each thread finds the first
// dynamic-Huffman block header in its range that decodes cleanly (a candidate), and decodes
// from there to the next thread's candidate, writing 16-bit symbols: a byte, or a reference
// to one of the 32768 bytes before its start that it cannot know yet.  The chain proves
// itself: the first range starts at the stream's start, and a range counts only when its
// decode ends on a block boundary exactly at the next range's candidate -- then that
// candidate is a real block start and the next range's decode is the stream's.  The
// references are resolved range by range from the previous range's last 32 KiB, the bytes
// land in one buffer, and the member's CRC-32 and size are checked.  Anything else (a
// candidate that was not a block start, a file with several members, a size past 4 GiB,
// too few candidates) returns false and the caller decodes the whole member on one thread.
#pragma once

#include <cstddef>
#include <cstdint>

namespace nw_gz {

struct Buffer {
    unsigned char* p = nullptr;   // mmap'd; release with release()
    size_t n = 0;                 // decompressed bytes
    size_t cap = 0;
    void release();
};

// crc32(buf) as zlib computes it, with libdeflate's folding implementation when the image
// has it (resolved by the caller: fn null -> zlib)
using Crc32Fn = uint32_t (*)(uint32_t, const void*, size_t);

// Decompresses the gzip file image [p, p + n) (one member) into *out with `threads` threads.
// false: not done (out empty) -- the caller takes the single-thread path, which also
// reports damaged data.
bool inflate_parallel(const unsigned char* p, size_t n, int threads, Crc32Fn crc, Buffer* out);

}  // namespace nw_gz
