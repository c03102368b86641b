// nw_device.h -- definitions shared by the HIP kernel and the host launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nw {

// Residue codes: 0..15 EDNAFULL (A T G C S W R Y K M B V H D N U),
// 16 = not in the matrix (scores 0 against everything).
constexpr int NCODE = 17;
constexpr int NCODE_PAD = 16;   // code used for columns past the end of a read

enum : int32_t { FLAG_EMPTY = 1 };

// Per-read record written by the kernel; layout matches nw_stat in include/crispr_nw.h.
struct Stat {
    int32_t aln_len, n_ident, n_sim, n_gaps, score, end_i, end_j, flags;
};

struct KernelArgs {
    const uint8_t* reads;      // packed read bytes
    const int64_t* offsets;    // n + 1 entries
    int64_t n;
    const int8_t* prof;        // [NCODE][64][RP] scaled EDNAFULL scores of each amplicon row
    const uint8_t* lut;        // [256] ascii -> code
    const uint8_t* amp;        // [La] amplicon bytes
    int32_t La;
    int32_t gap_open, gap_extend;   // scaled
    int32_t Lb_max;
    uint8_t* out;              // [n][3][stride]: aligned amplicon, markup, aligned read
    int64_t stride;
    Stat* stats;               // [n]
    uint8_t* tb_global;        // traceback slabs when they do not fit LDS
    int64_t tb_wave_bytes;
    int32_t debug_mode;        // 0 = normal; diagnostic builds of the phases: 1 = stop after
                               // the start-cell search, 2 = stop after the traceback walk
    // banded traceback storage (TB_BAND kernels)
    int32_t band_slots;        // columns of traceback kept per lane
    int64_t* fallback_list;    // reads whose traceback left the band are appended here
    int32_t* fallback_count;
    // work list (full-storage kernel re-running the fallbacks); null = all reads
    const int64_t* work_list;
    const int32_t* work_count;
    int32_t* work_counter;     // dynamic chunk queue of the pair kernel (zeroed per run)
};

// Traceback storage of a kernel instantiation.
enum TbMode : int { TB_LDS_FULL = 0, TB_GLOBAL_FULL = 1, TB_BAND = 2, TB_PAIR_BAND = 3 };

struct LaunchCfg {
    int R;           // amplicon rows per lane
    int wpb;         // waves per block
    int grid;        // blocks
    int lds_bytes;   // dynamic LDS per block
    int tb_mode;     // TbMode
};

int rows_per_lane_for(int La);
int profile_rp(int R);
int lds_bytes_for(int R, int La, int Lb_max, int tb_mode, int band_slots, int wpb);
int tb_bytes_per_wave(int R, int Lb_max);
hipError_t launch(const KernelArgs& a, const LaunchCfg& c, hipStream_t s);

// two-reads-per-wave packed int16 kernel (nw_pair.hip); band storage only.
// Blocks may hold up to kPairMaxThreads threads (its __launch_bounds__).
constexpr int kPairMaxThreads = 512;
int pair_lds_bytes_for(int R, int La, int Lb_max, int band_slots, int wpb);
int pair_profile_bytes_per_lane(int R);
hipError_t launch_pair(const KernelArgs& a, const LaunchCfg& c, hipStream_t s);

}  // namespace nw
