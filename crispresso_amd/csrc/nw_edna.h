// nw_edna.h -- EDNAFULL (NCBI NUC.4.4), the matrix EMBOSS needle scores with by
// default (CRISPRessoCORE.py:4226-4231 never sets -datafile).  Host side only:
// the kernels get it as score profiles / tables built by nw_host.cpp.
#pragma once
#include <cctype>
#include <cstdint>
#include <cstring>

namespace nw {

// order A T G C S W R Y K M B V H D N U
inline constexpr signed char kEdna[16][16] = {
    {5, -4, -4, -4, -4, 1, 1, -4, -4, 1, -4, -1, -1, -1, -2, -4},
    {-4, 5, -4, -4, -4, 1, -4, 1, 1, -4, -1, -4, -1, -1, -2, 5},
    {-4, -4, 5, -4, 1, -4, 1, -4, 1, -4, -1, -1, -4, -1, -2, -4},
    {-4, -4, -4, 5, 1, -4, -4, 1, -4, 1, -1, -1, -1, -4, -2, -4},
    {-4, -4, 1, 1, -1, -4, -2, -2, -2, -2, -1, -1, -3, -3, -1, -4},
    {1, 1, -4, -4, -4, -1, -2, -2, -2, -2, -3, -3, -1, -1, -1, 1},
    {1, -4, 1, -4, -2, -2, -1, -4, -2, -2, -3, -1, -3, -1, -1, -4},
    {-4, 1, -4, 1, -2, -2, -4, -1, -2, -2, -1, -3, -1, -3, -1, 1},
    {-4, 1, 1, -4, -2, -2, -2, -2, -1, -4, -1, -3, -3, -1, -1, 1},
    {1, -4, -4, 1, -2, -2, -2, -2, -4, -1, -3, -1, -1, -3, -1, -4},
    {-4, -1, -1, -1, -1, -3, -3, -1, -1, -3, -1, -2, -2, -2, -1, -1},
    {-1, -4, -1, -1, -1, -3, -1, -3, -3, -1, -2, -1, -2, -2, -1, -4},
    {-1, -1, -4, -1, -3, -1, -3, -1, -3, -1, -2, -2, -1, -2, -1, -1},
    {-1, -1, -1, -4, -3, -1, -1, -3, -1, -3, -2, -2, -2, -1, -1, -1},
    {-2, -2, -2, -2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -2},
    {-4, 5, -4, -4, -4, 1, -4, 1, 1, -4, -1, -4, -1, -1, -2, 5},
};
inline constexpr char kAlphabet[] = "ATGCSWRYKMBVHDNU";
constexpr int kCodeOther = 16;   // not in the matrix: scores 0 against everything

inline uint8_t code_of(unsigned char c) {
    const char* p = std::strchr(kAlphabet, std::toupper(c));
    return (c && p) ? (uint8_t)(p - kAlphabet) : (uint8_t)kCodeOther;
}

}  // namespace nw
