// wx_align.hip — MI355X (gfx950 / CDNA4) kernels for WhisperX's forced-alignment DP and
// VAD hysteresis, behind the C ABI of include/wx_align.h.
//
// Reference being replaced (file:line in NADOOIT/whisperX @ 2025-01-12):
//   get_trellis    whisperx/alignment.py:359-379     -> trellis_kernel (materialising)
//   backtrack      whisperx/alignment.py:387-421     -> bits_from_trellis_kernel + walk
//   merge_repeats  whisperx/alignment.py:438-454     -> merge_repeats_kernel
//   align() DP     whisperx/alignment.py:242-250     -> align_dp_kernel (fused, no trellis)
//   Binarize       whisperx/vad.py:118-180           -> binarize_kernel
//
// Design:
//   * One wave64 per segment.  The trellis recurrence is row-parallel: row t+1 depends only
//     on row t, so lane g owns the C contiguous cells j = g*C+1 .. g*C+C and a time step is
//     C independent add/add/max cells plus one DPP wave_shr:1 for the left neighbour of the
//     lane's first cell.  The sequential depth is T steps; throughput comes from many
//     segments (waves) in flight.
//   * Emission rows are staged 32 at a time into LDS (row stride VS = 32 or 64 floats) by
//     global_load_lds, double-buffered, so the per-cell gather em[t, tok[j-1]] is one
//     conflict-free ds_read_b32 with a compile-time immediate row offset.
//   * The fused kernel never writes the trellis.  The backtrack test at (t, j) is bit for
//     bit the forward comparison that produced trellis[t, j] (`changed > stayed`), so the
//     forward keeps one bit per cell per step: lane-local 32-step column words (v_cmp +
//     v_addc, shift-in), stored as [block][slot][lane].  The walk reads a 64-cell x 32-step
//     window of them per block into the wave's lanes and steps with v_readlane + scalar ops.
//   * merge_repeats is rebuilt from the walk's per-token start frames: token k spans
//     [start_k, start_{k+1}); its first frame carries exp(em[t, tok[k]]), the others
//     exp(em[t, 0]) (index 0, as alignment.py:409), summed left to right in fp64.
//
// Numerics are the reference's torch-CPU semantics (this file is compiled with
// -ffp-contract=off): fp32 adds, NaN-propagating max (v_maximum3_f32 == torch.maximum),
// strict `>` with ties staying, first-max/NaN-first argmax, fp64-accumulated column 0.
#ifndef WX_ALIGN_DP_H
#define WX_ALIGN_DP_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>

#include "../../include/wx_align.h"

#define WX_VERSION "0.1.0"

namespace wx {

constexpr int kWave = 64;
constexpr int kChunk = 32;  // emission rows per LDS buffer == bits per column word
constexpr int kUnroll = 8;  // time steps per unrolled group
constexpr int kMaxLdsFrames = 8192;  // segments up to this many frames keep walk state in LDS

template <bool B>
struct BoolTag {
    static constexpr bool value = B;
};

__device__ __forceinline__ float nan_max(float a, float b) {
    // IEEE-754-2019 maximum (NaN-propagating): torch.maximum for non-zero-sign cases.
    return __builtin_elementwise_maximum(a, b);
}

// w <- 2w + (c > s): strict compare (false when unordered), shifted into the lane's
// 32-step column word with an add-with-carry.
__device__ __forceinline__ unsigned shift_in(unsigned w, float c, float s) {
    unsigned r;
    asm("v_cmp_gt_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %3, %3, vcc"
        : "=v"(r)
        : "v"(c), "v"(s), "v"(w)
        : "vcc");
    return r;
}


// Correctly rounded fp32 exp (the reference's torch-CPU exp is within 1 ULP of it).
__device__ __forceinline__ float exp_cr(float x) { return (float)exp((double)x); }

__device__ __forceinline__ float dpp_shr1(float old_lane0, float v) {
    // lane l <- v[l-1]; lane 0 keeps old_lane0 (bound_ctrl off).
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old_lane0), __builtin_bit_cast(int, v),
                                           0x138 /* wave_shr:1 */, 0xF, 0xF, false));
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uniform64(int64_t x) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(uint64_t)x);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float uniformf(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
// lane l's 64-bit value, wave-uniform (two v_readlane)
__device__ __forceinline__ unsigned long long readlane64(unsigned long long x, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// Column 0's running sum over one 32-row chunk (alignment.py:366-370: torch's CPU cumsum
// accumulates em[:, 0] in double, row by row).  Lane j converts em[t0 + j, 0] (one instruction
// for the chunk), the doubles go through LDS and come back broadcast (16-byte reads, every lane
// the same address), and at step j the lanes r > j add row j: an EXEC-masked v_add_f64 with a
// scalar s_bitset0 retiring lane j + 1 after it.  Lane r (0..32) thus adds em[t0 + 0 .. r - 1, 0]
// in row order onto S(t0) and nothing else — the sequential chain's additions exactly.  (Round
// 5: two instructions per row instead of a conversion, a DPP shift and the add; config 2 50.8
// -> 47.5 us.)
__device__ __forceinline__ double col0_chain(double acc, float e) {
    const int l = lane_id();
    __shared__ __attribute__((aligned(16))) double c0d[kChunk];
    if (l < kChunk) c0d[l] = (double)e;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (other lanes' writes, read below)
    double dv[kChunk];
#pragma unroll
    for (int j = 0; j < kChunk; ++j) dv[j] = c0d[j];
    double a = acc;
    unsigned long long sv;
#define WX_C0_STEP(J, BIT) "v_add_f64 %[a], %[a], %[d" #J "]\n\ts_bitset0_b64 exec, " #BIT "\n\t"
#define WX_C0_BLOCK(B, J0, B1, B2, B3, B4, B5, B6, B7, B8)                                                      \
    asm volatile("s_mov_b64 %[sv], exec\n\t"                                                                  \
                 "s_mov_b32 exec_lo, %[mlo]\n\t"                                                              \
                 "s_mov_b32 exec_hi, 1\n\t" WX_C0_STEP(0, B1) WX_C0_STEP(1, B2) WX_C0_STEP(2, B3)              \
                     WX_C0_STEP(3, B4) WX_C0_STEP(4, B5) WX_C0_STEP(5, B6) WX_C0_STEP(6, B7)                   \
                         WX_C0_STEP(7, B8) "s_mov_b64 exec, %[sv]\n\t"                                        \
                 : [a] "+v"(a), [sv] "=&s"(sv)                                                                 \
                 : [mlo] "s"((unsigned)(0xFFFFFFFFu << ((J0) + 1))), [d0] "v"(dv[(J0)]),                      \
                   [d1] "v"(dv[(J0) + 1]), [d2] "v"(dv[(J0) + 2]), [d3] "v"(dv[(J0) + 3]),                     \
                   [d4] "v"(dv[(J0) + 4]), [d5] "v"(dv[(J0) + 5]), [d6] "v"(dv[(J0) + 6]),                     \
                   [d7] "v"(dv[(J0) + 7]))
    // block b: rows 8b .. 8b + 7, lanes 8b + 1 .. 32 active at its start (exec_hi = lane 32)
    WX_C0_BLOCK(0, 0, 1, 2, 3, 4, 5, 6, 7, 8);
    WX_C0_BLOCK(1, 8, 9, 10, 11, 12, 13, 14, 15, 16);
    WX_C0_BLOCK(2, 16, 17, 18, 19, 20, 21, 22, 23, 24);
    WX_C0_BLOCK(3, 24, 25, 26, 27, 28, 29, 30, 31, 32);
#undef WX_C0_BLOCK
#undef WX_C0_STEP
    return a;
}

// One chunk of column 0's running sum: lane l (0..31) holds e = em[t0 + l, 0] (lanes 32..63:
// any copy), acc = S(t0) (uniform).  Returns S(t0 + l) on lane l and advances acc to S(t0 + 32)
// (lane 32's sum, by v_readlane: no LDS round trip).
__device__ __forceinline__ double col0_chunk(double& acc, float e) {
    const double a = col0_chain(acc, e);
    acc = __builtin_bit_cast(double, readlane64(__builtin_bit_cast(unsigned long long, a), kChunk));
    return a;
}

// Cell values live in an ext_vector so that the one dynamic (wave-uniform) index of the
// step — the slot holding column N — lowers to s_set_gpr_idx_on/v_mov instead of scratch.
template <int C>
using cellvec = float __attribute__((ext_vector_type(C)));

struct SegDesc {
    int64_t row0;  // first emission row
    int T;
    int64_t tok0;
    int N;
    int blank;
};

__device__ __forceinline__ SegDesc load_desc(const int64_t* em_off, const int64_t* tok_off, const int32_t* blank_id,
                                             int seg) {
    SegDesc d;
    d.row0 = em_off[seg];
    d.T = uniform((int)(em_off[seg + 1] - d.row0));
    d.tok0 = tok_off[seg];
    d.N = uniform((int)(tok_off[seg + 1] - d.tok0));
    d.blank = uniform(blank_id[seg]);
    return d;
}

// LDS byte address of a __shared__ pointer (for M0).
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// Wave-uniform 64-bit pointer (SGPR pair).
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// LDS-DMA loads (global_load_lds), saddr form: wave-uniform base + 32-bit lane offset
// (inline-asm 64-bit VGPR operands are not guaranteed the even alignment gfx950 requires).
// Lane l's dword (or 16 bytes) lands at LDS m0 + 4*l (16*l).  Issued from inline asm so
// that hipcc's waitcnt pass does not see them (it would otherwise drain vmcnt before every
// ds_read, serialising the prefetch); callers wait vmcnt(0) themselves before reading.
__device__ __forceinline__ void glds_dword(const float* sbase, unsigned voff, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(uniform_ptr(sbase)), "s"(lds_dst)
                 : "memory");
}
// ... with device scope (sc1): the hand-off granules another CU writes (granule_load's scope)
__device__ __forceinline__ void glds_dwordx4_sc1(const void* sbase, unsigned voff, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(uniform_ptr((const float*)sbase)), "s"(lds_dst)
                 : "memory");
}
__device__ __forceinline__ void glds_dwordx4(const float* sbase, unsigned voff, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(uniform_ptr(sbase)), "s"(lds_dst)
                 : "memory");
}

// Large vocabularies (V > 64, e.g. ja/zh character sets): the DP reads only column 0, the
// blank and the segment's own tokens, so a per-segment column map (built in LDS by
// build_colmap) lets the staging gather exactly those columns into a compact LDS row of
// VS = kGatherVS floats.  Token ids are remapped to their compact rank.
constexpr int kGatherVS = 256;                      // compact row width (distinct columns)
constexpr int kMaxVocabWords = WX_MAX_VOCAB / 32;   // used-column bitmap words

struct ColMap {
    const unsigned* bm;  // LDS: used-column bitmap
    const int* wpre;     // LDS: set bits in the words before each word
    const int* cols;     // LDS: compact index -> column
    int n;               // compact width (uniform)
    __device__ __forceinline__ int rank(int c) const {
        const int w = c >> 5;
        return wpre[w] + __popc(bm[w] & ((1u << (c & 31)) - 1u));
    }
};

// Stage emission rows [r0, r0+nrows) of a segment into LDS buffer `dst` (row stride VS
// floats).  Every wave of the workgroup issues its share.  When V == VS == 32 and the
// rows are 16-byte aligned (`x4`), a chunk is one contiguous 4 KB block in both places:
// one 16-byte-per-lane instruction moves 8 rows.  VS == kGatherVS: per row, lane l of pass
// i gathers column cols[64i + l] (the LDS-DMA source address is per lane, the destination
// lane-linear).  Otherwise one dword per lane per row, lanes >= V masked.  Asynchronous:
// every wave waits vmcnt(0) before the chunk barrier.
template <int VS, int W, bool ONE_WAVE = false>
__device__ __forceinline__ void stage_rows(const float* __restrict__ E, int V, int r0, int nrows, float* dst,
                                           bool x4, const ColMap& cm) {
    const int wv = ONE_WAVE ? 0 : uniform((int)threadIdx.x >> 6);
    const int l = lane_id();
    const unsigned base = (unsigned)uniform((int)lds_addr(dst));
    if (VS == kGatherVS) {
        const int passes = (cm.n + kWave - 1) / kWave;
        for (int i = 0; i < passes; ++i) {
            const int c = i * kWave + l;
            if (c < cm.n) {
                const unsigned off = (unsigned)cm.cols[c] * 4u;
                for (int r = wv; r < nrows; r += W)
                    glds_dword(E + (int64_t)(r0 + r) * V, off, base + (unsigned)(r * VS * 4 + i * kWave * 4));
            }
        }
    } else if (VS == 32 && x4) {
        for (int i = wv; i * 8 < nrows; i += W) {
            if (i * 8 + (l >> 3) < nrows)
                glds_dwordx4(E + (int64_t)(r0 + i * 8) * 32, (unsigned)l * 16u, base + (unsigned)(i * 1024));
        }
    } else if (l < V) {
        for (int r = wv; r < nrows; r += W)
            glds_dword(E + (int64_t)(r0 + r) * V, (unsigned)l * 4u, base + (unsigned)(r * VS * 4));
    }
}

// Quad-interleaved staging (the register-resident forward, Forward::kReg).  A chunk's 32 rows
// are kept as 8 row quads; quad p holds, per column c, the 4 values em[4p..4p+3, c] in 16
// contiguous bytes: float index p * QS + 4 c + (row & 3), QS = 4 (VS + 1).  One 16-byte LDS
// read then gives a lane 4 steps of its token's column (and, read at a uniform address, 4
// steps of the blank), instead of one or two dwords per step.  Column VS of each quad is not
// staged: the column-0 helper writes the column-1 wave's lane-0 operand there (see
// Forward::col0_pre).  The stager fills it from a row-major LDS-DMA ring (Forward::transpose_quads).
template <int VS>
__host__ __device__ constexpr int quad_stride() { return 4 * (VS + 1); }
template <int VS>
__host__ __device__ constexpr int quad_buf_floats() { return 8 * quad_stride<VS>(); }

// The column map of one segment (all threads of the workgroup): columns 0 and `blank` and
// every token id (ids outside [0, V) count as 0, as the DP reads them).  Returns the compact
// width, uniform; > kGatherVS means the segment cannot be staged.
__device__ int build_colmap(const int32_t* __restrict__ tok, int N, int blank, int V, unsigned* bm, int* wpre,
                            int* cols) {
    const int nw = (V + 31) >> 5;
    for (int w = (int)threadIdx.x; w < nw; w += (int)blockDim.x) bm[w] = 0u;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int b = (blank >= 0 && blank < V) ? blank : 0;
        atomicOr(&bm[0], 1u);
        atomicOr(&bm[b >> 5], 1u << (b & 31));
    }
    for (int j = (int)threadIdx.x; j < N; j += (int)blockDim.x) {
        int t = tok[j];
        t = (t >= 0 && t < V) ? t : 0;
        atomicOr(&bm[t >> 5], 1u << (t & 31));
    }
    __syncthreads();
    if (threadIdx.x < kWave) {  // exclusive prefix of popcounts, 64 words per pass
        int base = 0;
        for (int w0 = 0; w0 < nw; w0 += kWave) {
            const int w = w0 + (int)threadIdx.x;
            const int c = w < nw ? __popc(bm[w]) : 0;
            int incl = c;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const int y = __shfl_up(incl, off);
                if ((int)threadIdx.x >= off) incl += y;
            }
            if (w < nw) wpre[w] = base + incl - c;
            base += __shfl(incl, kWave - 1);
        }
        if (threadIdx.x == 0) wpre[nw] = base;
    }
    __syncthreads();
    const int n = wpre[nw];
    if (n <= kGatherVS) {
        for (int w = (int)threadIdx.x; w < nw; w += (int)blockDim.x) {
            unsigned m = bm[w];
            int k = wpre[w];
            while (m) {
                cols[k++] = w * 32 + __ffs((int)m) - 1;
                m &= m - 1u;
            }
        }
    }
    __syncthreads();
    return uniform(n);
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wave_fence() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void block_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Column-0 value tr[t][0]: 0 / fp32(cumsum) / +inf in the last N rows (alignment.py:367-370).
__device__ __forceinline__ float col0_value(int t, double acc, int T, int N) {
    const bool inf_row = (N == 0) || (t >= T + 1 - N);
    if (inf_row) return INFINITY;
    return t == 0 ? 0.0f : (float)acc;
}

// ------------------------------------------------------------------------------------
// Cell -> (lane, slot) layout of one segment.  G = ceil(N/C) lanes are used; the first
// n_short of them own C-1 cells, the rest C cells, so that column N always sits in the
// compile-time slot C-1 of lane G-1 (its value feeds the argmax every step without a
// dynamic register index).  Lanes >= G and the spare slot C-1 of short lanes compute
// harmless garbage: cells only ever feed cells to their right.
struct Layout {
    int C;        // cells per full lane
    int G;        // lanes used
    int n_short;  // leading lanes with C-1 cells
    int lanes;    // lanes of the workgroup (bitmap word stride)

    __host__ __device__ static Layout make(int C, int N, int lanes) {
        Layout L;
        L.C = C;
        L.lanes = lanes;
        L.G = (N + C - 1) / C;
        const int n_full = N - L.G * (C - 1);
        L.n_short = L.G - n_full;
        return L;
    }
    // first cell (1-based) and cell count of lane g
    __device__ __forceinline__ int first(int g) const {
        return g < n_short ? g * (C - 1) + 1 : n_short * (C - 1) + (g - n_short) * C + 1;
    }
    __device__ __forceinline__ int count(int g) const { return g < n_short ? C - 1 : (g < G ? C : 0); }
    // (lane, slot) of 0-based cell c; CC = C when known at compile time (0: runtime C)
    template <int CC = 0>
    __device__ __forceinline__ void locate(int c, int& g, int& k) const {
        const int Cc = CC > 0 ? CC : C;
        const int cs = n_short * (Cc - 1);
        if (c < cs) {
            g = Cc > 1 ? c / (Cc - 1) : 0;
            k = c - g * (Cc - 1);
        } else {
            const int c2 = c - cs;
            g = n_short + c2 / Cc;
            k = c2 - (g - n_short) * Cc;
        }
    }
};

// ------------------------------------------------------------------------------------
#ifdef WX_PHASE_TIMING
// Debug build only: per-segment s_memtime at kernel entry / forward end / walk end / exit,
// plus s_memrealtime at entry and exit (100 MHz) to convert cycles to time.
__device__ unsigned long long wx_phase[8192 * 6];
// per (segment, wave): cycles in steps / barrier waits / other chunk work
constexpr int kLoopSlots = 32;  // per workgroup, 3 counters each
__device__ unsigned long long wx_loop[8192 * kLoopSlots * 3];
// per (workgroup, chunk): s_memrealtime when wave 0 passed barrier q, when wave W-1 stored
// chunk q's halo granules, when wave 0 had chunk q's halo (split kernels)
__device__ unsigned long long wx_cq[8192 * 48 * 3];
#define WX_CQ(q, i) \
    if (lane_id() == 0 && blockIdx.x < 8192 && (q) < 48) wx_cq[(blockIdx.x * 48 + (q)) * 3 + (i)] = __builtin_amdgcn_s_memrealtime()
#define WX_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define WX_STAMP(i) \
    if (threadIdx.x == 0 && blockIdx.x < 8192) wx_phase[blockIdx.x * 6 + (i)] = __builtin_amdgcn_s_memtime()
#define WX_STAMP_RT(i) \
    if (threadIdx.x == 0 && blockIdx.x < 8192) wx_phase[blockIdx.x * 6 + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define WX_STAMP(i)
#define WX_STAMP_RT(i)
#define WX_T(v)
#define WX_CQ(q, i)
#endif

// The trellis forward pass shared by the fused and the materialising kernels.
//   MODE 0: fused — per-cell 32-step decision words -> bits, column N history -> cn.
//   MODE 1: materialise — write every trellis row (get_trellis).
//   MODE 2: checkpointed — no decision bits: at each chunk start (row 32q) every owner lane
//           stores its C cell values in the bitmap's word layout, and wave 0 the fp64
//           column-0 cumsum; the walk recomputes each block's band from them (CkSrc).  A
//           cell step is then 3 VALU (add, DPP add, maximum) instead of 5.
//
// W > 1 waves split the columns of one segment with a chunk halo instead of a per-step
// exchange: wave w >= 1 spends its first HL = ceil(32/C) lanes re-computing the last HL
// lanes of wave w-1 (>= 32 cells).  At each chunk start (row 32q) those cells are copied
// from wave w-1 through LDS; during the chunk's 32 steps the wrong value that enters at
// the halo's left edge moves right by one cell per step, so it never reaches the wave's
// own cells (cell j at row t depends only on cells j-s..j at row t-s).  The waves meet
// once per chunk at the barrier that also publishes the staged emission rows.  Halo lanes
// compute bit-identical copies (same operands, same order) and only the owning lane
// writes decisions / trellis values.
//
// H (helper): one more wave per workgroup stages the emission rows two chunks ahead and
// computes column 0 (the fp64 cumsum, +inf rows) and q0 = exp(em[t,0]) one chunk ahead, so
// the column-1 wave reads column 0 from LDS instead of running the fp64 chain per step.
// Split segments (latency mode, few segments): one segment's columns are spread over P
// workgroups ("parts", one per CU), continuing the chunk halo across CUs.  Virtual wave
// vw = part * W + wv; the first HL lanes of a part's wave 0 mirror the last HL lanes of
// the previous part's wave W-1, handed over once per 32-row chunk through global memory
// as 8-byte {value, tag} granules (one sc1 store each; the tag is the launch's 32-bit epoch and
// each chunk has its own slot, so a granule is valid on its own — no flag, no fence; the
// region is zeroed before first use and holds only granules, so a stale word carries an older
// launch's epoch and never matches).  A part lags its
// predecessor by a few chunks; the consumer prefetches each chunk's granules two chunks
// ahead.  Each part then arrives at a per-segment counter;
// the last to arrive runs the argmax, the walk and merge_repeats.
constexpr int kMaxParts = 4;
// Column-N history: segment s at (row0 + kCnPad s) rounded down to 16 bytes, so at least
// kCnPad - 3 floats past its T rows are its own: the register-resident owner stores all four
// 8-row groups of a partial last chunk, up to 31 rows past T.
constexpr int kCnPad = 40;
constexpr int kXcdStride = 8;  // blocks b and b + 8 share an XCD (MI355X: 8 XCDs, round-robin)
__host__ __device__ constexpr unsigned split_grid(int S, int P) {
    return (unsigned)((S + kXcdStride - 1) / kXcdStride * kXcdStride * P);
}
constexpr int kHaloCells = 40;  // >= HL * C = ceil(32 / C) * C for every C
constexpr int kMaxSpin = 1 << 16;
constexpr int kXSlack = 1;  // chunks a part re-builds its lag to (A/B: 1 >= 2 > 3 > 4)

struct Split {
    int p, P;         // this part, parts per segment
    int lanes;        // bitmap word stride: 64 * W * P
    unsigned tag;     // the launch epoch (32 bits, never 0)
    uint64_t* xin;    // granules from part p-1: [chunk][kHaloCells] (p > 0)
    uint64_t* xout;   // granules to part p+1 (p < P-1)
    int xstride;      // granules per chunk block of one segment boundary
    int spin;         // re-reads before a hand-off counts as lost (kMaxSpin; 0 in the recovery test)
    // Register-resident kernels: the idle helper wave of a part > 0 polls the granules of
    // chunk q and leaves their values in xg[q & 1] before barrier q; the hand-off consumer (DP
    // wave 0) reads them there after the barrier like any other wave's halo, so no DP wave
    // issues a global load.  (Routed through the consumer itself — prefetches two chunks ahead
    // by LDS-DMA, hand-counted vmcnt, its bitmap stores handed to the helper — every missed
    // prefetch cost a round trip inside the chain and the parts drifted apart: 59.7 us.)
    float* xg;  // LDS [2][32]
    float* q0l;  // LDS [T]: q0 = exp(em[t, 0]), filled by the extra walker waves (nullptr: not kept)
};

__device__ __forceinline__ void granule_store(uint64_t* g, float v, unsigned tag) {
    const uint64_t x = ((uint64_t)tag << 32) | (uint64_t)__builtin_bit_cast(unsigned, v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store_dwordx2 sc1
}
__device__ __forceinline__ uint64_t granule_load(const uint64_t* g) {
    return __hip_atomic_load(const_cast<uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Split segments publish their decision words and column-N history write-through (WT: sc1
// stores, which leave the XCD's L2 at once) and the last part to arrive reads them with sc1
// loads, L1-bypassing: the arrival then needs neither the release fence (buffer_wbl2: the
// write-back of every dirty line of the XCD's L2, ~2-6 us behind a part's freshly written
// bits) nor the acquire (MI355X_MICROARCH.md, "Valid forms": one lane per storing workgroup
// adds to one counter after every storing wave's vmcnt(0) wait and a workgroup barrier, the
// workgroup whose add came last loads after it returned, its other waves after a barrier;
// 4- and 16-byte sc1 stores and loads).  That table is measured behaviour on gfx950 / ROCm
// 7.2 (the guide's hand-off table, row 1), not an architectural guarantee, so the launch flag
// kArgFenced (WX_SPLIT_FENCED=1) adds the agent-scope release and acquire on top of the
// write-through stores — the memory model's own protocol — and the parity tests compare the
// two bit for bit with the parts of every segment spread over different XCDs (kArgXcdSpread).
constexpr bool kSplitWT = true;
constexpr int kArgFenced = 1;     // AlignArgs::flags: release/acquire at the split arrival
constexpr int kArgXcdSpread = 2;  // AlignArgs::flags: parts of a segment on different XCDs (tests)
// Register-resident split kernels only (C = 1, config 2): in the C > 1 split kernels the
// consumer's hand-off waits drain vmcnt inside the chain, and write-through stores take longer
// to drain (A/B, 64 x T = 2999, N ~ 900: fenced 166 us, write-through 178 us).
template <int C, int VS, bool SP>
constexpr bool split_wt() {
    return SP && kSplitWT && C == 1 && VS != kGatherVS;
}
template <bool WT, class T>
__device__ __forceinline__ T ld_pub(const T* p) {
    if constexpr (WT)
        return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load_dword sc1
    else
        return *p;
}
template <bool WT, class T>
__device__ __forceinline__ void st_pub(T* p, T v) {
    if constexpr (WT)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store_dword sc1
    else
        *p = v;
}
// 16 bytes at base[i .. i + 3] (base wave-uniform).  WT: a buffer store with the sc1 bit (aux
// 16), through the builtin so that the compiler keeps its hazard and vmcnt bookkeeping (an asm
// dwordx4 store's data registers could be overwritten in the next instruction).
template <bool WT>
__device__ __forceinline__ void st_pub4(float* base, int i, float4 v) {
    if constexpr (WT) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
        const u4 x = {__builtin_bit_cast(unsigned, v.x), __builtin_bit_cast(unsigned, v.y),
                      __builtin_bit_cast(unsigned, v.z), __builtin_bit_cast(unsigned, v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(x, r, i * 4, 0, 16);
    } else {
        *reinterpret_cast<float4*>(base + i) = v;
    }
}

template <int C, int W>
struct Geometry {
    static constexpr int HL = W > 1 ? (32 + C - 1) / C : 0;  // halo lanes per wave >= 1
    static constexpr int kUseful = kWave + (W - 1) * (kWave - HL);  // useful lanes
    static constexpr int kCapacity = C * kUseful;                   // max N
    // useful lane index of (wave, lane); for a halo lane, the lane it mirrors
    __host__ __device__ static constexpr int lane_of(int wv, int l) {
        return wv == 0 ? l : kWave + (wv - 1) * (kWave - HL) + l - HL;
    }
    // (wave, lane) owning useful lane g
    __device__ static void owner(int g, int& wv, int& l) {
        if (g < kWave || W == 1) {
            wv = 0;
            l = g;
        } else {
            wv = 1 + (g - kWave) / (kWave - HL);
            l = HL + (g - kWave) % (kWave - HL);
        }
    }
};

template <int C, int VS, int MODE, int W, bool H, bool SP = false, int NH = 1>
struct Forward {
    static constexpr int kRowBytes = VS * 4;
    static constexpr int kLanes = kWave * W;  // bitmap word stride (DP waves; SP: Split::lanes)
    // emission chunk buffers in LDS; kReg (declared below) keeps five: its helper restages
    // chunk q + 4 at barrier q into the buffer of chunk q - 1, the newest one no wave may still
    // be reading (the DP waves read chunk q's operands until chunk q's first step, after
    // barrier q — chunk 0's only after barrier 0)
    static constexpr int kBufs = (C == 1 && MODE == 0 && SP && NH == 2 && VS != kGatherVS) ? 5 : (H ? 4 : 2);
    // Software-pipelined LDS operands where the extra registers keep the occupancy that
    // matters: latency buckets (2 waves per SIMD by design) and one-wave buckets up to
    // C = 8; the multi-wave C = 8 buckets lose a wave per SIMD to them (A/B: -17%).
    static constexpr bool kPipelined = H || (MODE != 1 && (C <= 6 || (C == 8 && W == 1)));
    // Column 0 (tr[t][0]) read from LDS by the column-1 wave (COL kColLds): the helper wave
    // computes it (H), or — checkpointed multi-wave kernels — DP wave 1 does, a chunk ahead
    // (c0_make): the fp64 cumsum per step otherwise paced wave 0 (+25% steps in the phase timing).
    static constexpr bool kC0Lds = H || (MODE == 2 && W >= 2);
    using Geo = Geometry<C, (SP ? 2 : W)>;  // SP: always a halo (the waves span P parts)
    // Steps per unrolled group of the non-pipelined chunk (hipcc hoists the group's LDS
    // loads; a multiple of 4: column-N history is stored as float4).
    static constexpr int kU = kUnroll;
    static_assert(!(H && MODE == 1), "the materialising kernel computes column 0 in wave 0");
    // Register-resident chunks (split kernels with one cell per lane, the latency shape of
    // config 2): a chunk's operands are read into registers during the previous chunk (16-byte
    // reads of quad-interleaved rows), so the 32 steps of a chunk are a pure VALU chain — no
    // LDS read, no wait.  Micro-benchmarks (tools/ubench/step*.hip): a step costs ~20 cycles
    // of one wave alone, each LDS read issued inside the chain ~9 more.
    static constexpr bool kReg = C == 1 && MODE == 0 && SP && NH == 2 && VS != kGatherVS;
    static constexpr bool kWT = split_wt<C, VS, SP>();
    static constexpr int kBufFloats = kReg ? quad_buf_floats<VS>() : kChunk * VS;  // one chunk buffer
    static constexpr int kQS = quad_stride<VS>();

    // Per-lane state of the forward pass.
    struct State {
        cellvec<C> cur;
        unsigned w[C];
        double acc;   // W == 1 / !H: column-0 cumsum (fp64)
        float col0;   // tr[t][0] for the current step (column-1 wave)
        int t;
        // MODE 1 row stores, transposed through LDS so that every global store instruction
        // writes 256 contiguous bytes of the row: lane l stores the wave's own cells
        // jbase + l + 64 i, read from the wave's staging row at rd[i] (-1: none).
        float* rs;
        int jbase;
        int rd[C];
    };

    // SP: make xpre[] hold chunk q's halo granules (lanes < HL, C each), re-reading until
    // every tag matches.  Returns whether they were already there; bounded (sets lost).
    __device__ __forceinline__ static bool xwait(const uint64_t* xin, int xstride, int q, int l, unsigned tag,
                                                 uint64_t (&xpre)[C], bool& lost, int spin) {
        constexpr int HL = Geometry<C, 2>::HL;
        const unsigned want = tag;  // the slot already encodes the chunk; the tag is the launch
        const uint64_t* gi = xin + (int64_t)q * xstride + min(l, HL - 1) * C;  // all lanes load
        bool ok = true;
#pragma unroll
        for (int k = 0; k < C; ++k) ok = ok && (l >= HL || (unsigned)(xpre[k] >> 32) == want);
        const bool first = __all(ok);
        if (!first) {
            for (int it = 0; !lost && !__all(ok) && it < spin; ++it) {
                __builtin_amdgcn_s_sleep(2);
                ok = true;
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    xpre[k] = granule_load(gi + k);
                    ok = ok && (l >= HL || (unsigned)(xpre[k] >> 32) == want);
                }
            }
            // The re-read loop issues a data-dependent number of loads: end it with nothing in
            // flight, so that hipcc's waitcnt analysis still knows how many loads are pending
            // at the next chunk's check and waits for the two-chunk-old prefetch only (an
            // unbounded count made it wait vmcnt(0) there: the prefetch issued one chunk ago
            // and the previous chunk's bitmap stores were waited for at every chunk).
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        lost = lost || !__all(ok);
        return first;
    }

    // All waves of the workgroup call run(); with H, wave W is the helper.
    __device__ __forceinline__ static bool run(const SegDesc& d, const float* __restrict__ E, int V,
                                               const int32_t* __restrict__ tok,
                                               unsigned* __restrict__ bits,  // MODE 0: segment's bitmap
                                               float* __restrict__ q0,        // MODE 0: exp(em[t,0]) per row
                                               float* __restrict__ cn,        // MODE 0: column N of rows 1..T
                                               float* __restrict__ tr,        // MODE 1: trellis
                                               float* lds /* kBufs * kBufFloats */,
                                               float* c0b /* H: 2 * kChunk column-0 values */,
                                               float* xh /* 2 * W * 64: chunk halo copies */, bool x4,
                                               const ColMap& cm /* VS == kGatherVS: column map */,
                                               float* rst = nullptr /* MODE 1: W * 64 * C row staging */,
                                               const Split* sp = nullptr /* SP */,
                                               double* c0acc = nullptr /* MODE 2: column-0 cumsum per chunk */) {
        const int wv = uniform((int)threadIdx.x >> 6);
        const int vw = SP ? sp->p * W + wv : wv;  // virtual wave (SP: across parts)
        const int lanes = SP ? sp->lanes : kLanes;
        const int T = d.T, N = d.N;
        const int nch = (T + kChunk - 1) / kChunk;
        // checkpointed multi-wave kernels: wave 1 makes column 0 of chunk q + 1 (into c0b, and
        // its cumsum at row 32 (q + 1) into c0acc) after its chunk-q steps, from em[., 0] loaded a
        // chunk ahead: the kReg helper's lane-parallel, order-preserving fp64 prefix (col0_pre)
        const bool c0prod = MODE == 2 && W >= 2 && wv == 1;
        double c0a = 0.0;  // S(32 q) of the next chunk to make (uniform)
        float c0e = 0.0f;
        const int l0 = lane_id();
        auto c0_load = [&](int qq) { return E[(int64_t)min(qq * kChunk + (l0 & 31), T - 1) * V]; };
        auto c0_make = [&](int qq, float e) {
            float x = l0 >= 32 ? e : 0.0f;
            double a = c0a;
#pragma unroll
            for (int j = 0; j < kChunk; ++j) {
                a += (double)x;
                x = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x130 /* wave_shl:1 */,
                                                                       0xF, 0xF, true));
            }
            if (l0 == 0) c0acc[qq] = c0a;
            if (l0 < kChunk) c0b[(qq & 1) * kChunk + l0] = col0_value(qq * kChunk + l0, a, T, N);
            c0a = __shfl(a, kChunk);
        };
        if (c0prod && nch > 0) c0_make(0, c0_load(0));  // (before barrier 0)
        if (H && wv >= W + NH) {
            // split kernels' extra walker waves: keep the barrier count, and meanwhile fill
            // q0 = exp(em[t, 0]) (alignment.py:409's stay probabilities) into this part's LDS for
            // merge_repeats — the last part to arrive then has it at hand (fill_q0 after the walk
            // was ~1 us of config 2's tail).  64 rows per wave and chunk, loaded two chunks ahead
            // (unconditional, clamped), so no barrier waits on a load.
            float* q0l = SP ? sp->q0l : nullptr;
            const int nxw = (int)(blockDim.x >> 6) - W - NH;
            const int step = kWave * nxw;
            const int l = lane_id();
            int r0 = (wv - W - NH) * kWave;  // (uniform) first row of this wave's current group
            float e0 = 0.0f, e1 = 0.0f;
            if (q0l) {
                e0 = E[(int64_t)min(r0 + l, T - 1) * V];
                e1 = E[(int64_t)min(r0 + step + l, T - 1) * V];
            }
            if (kReg) __syncthreads();  // (barrier -1)
            for (int q = 0; q < nch; ++q) {  // 64 nxw rows per chunk of 32 rows: done by chunk nch / 2
                __syncthreads();
                if (q0l && r0 < T) {
                    if (r0 + l < T) q0l[r0 + l] = exp_cr(e0);
                    e0 = e1;
                    r0 += step;
                    e1 = E[(int64_t)min(r0 + step + l, T - 1) * V];
                }
            }
            return false;
        }
        if (H && wv >= W) {
            // NH == 2 (split kernels): wave W stages, wave W + 1 runs column 0's fp64 chain;
            // one helper doing both paced part 0 (it reached every chunk barrier last)
            const bool col0 = (!SP || sp->p == 0) && (NH == 1 || wv == W + 1);
            if constexpr (kReg) {
                int t0 = N > 0 ? tok[d.tok0] : 0;
                t0 = (t0 >= 0 && t0 < V) ? t0 : 0;
                return helper_reg(d, E, V, lds, lds + kBufs * kBufFloats, nch, t0, col0, wv == W, x4, sp);
            } else {
                helper(d, E, V, lds, c0b, nch, x4, cm, col0, NH == 1 || wv == W);
            }
            return false;
        }
        const int l = lane_id();
        const Layout L = Layout::make(C, N, lanes);
        if (MODE == 1) {
            if (threadIdx.x == 0) tr[0] = col0_value(0, 0.0, T, N);
            for (int j = (int)threadIdx.x + 1; j <= N; j += kLanes) tr[j] = -INFINITY;
        }
        if ((W > 1 || SP) && vw > 0 && Geo::lane_of(vw, Geo::HL) >= L.G) {
            // no column of this wave exists: keep the barrier count (and, without a helper,
            // this wave's share of the staging)
            if (!H && nch > 0) stage_rows<VS, W>(E, V, 0, min(kChunk, T), lds, x4, cm);
            if (kReg) __syncthreads();  // (the register-resident protocol's barrier -1)
            for (int q = 0; q < nch; ++q) {
                wait_vm();
                __syncthreads();
                if (c0prod && q + 1 < nch) c0_make(q + 1, c0_load(q + 1));
                if (!H && q + 1 < nch)
                    stage_rows<VS, W>(E, V, (q + 1) * kChunk, min(kChunk, T - (q + 1) * kChunk),
                                      lds + ((q + 1) % kBufs) * kBufFloats, x4, cm);
            }
            return false;
        }
        const int g = Geo::lane_of(vw, l);  // useful lane this lane computes
        const bool halo = vw > 0 && l < Geo::HL;
        // SP: wave W-1 hands its last HL lanes to the next part (if that part has columns);
        // wave 0 of parts > 0 takes its halo lanes from the previous part.
        const bool xpub = SP && wv == W - 1 && sp->p + 1 < sp->P && Geo::lane_of(vw + 1, Geo::HL) < L.G;
        const bool xsub = SP && wv == 0 && sp->p > 0;
        // (own_w, own_l below: column N's wave and lane)
        const int f = L.first(g), cnt = L.count(g);
        const bool is_short = g < L.n_short;
        // per-slot LDS byte offsets of em[., tok[j-1]]
        int toff[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int j = f + k;
            int tk = (k < cnt && j <= N) ? tok[d.tok0 + j - 1] : 0;
            tk = (tk >= 0 && tk < V) ? tk : 0;
            toff[k] = (VS == kGatherVS ? cm.rank(tk) : tk) * 4;
        }
        const int boff = (VS == kGatherVS ? cm.rank(d.blank) : d.blank) * 4;  // column 0 has rank 0
        // column N = slot C-1 of useful lane G-1
        int own_w, own_l;
        Geo::owner(L.G - 1, own_w, own_l);
        const bool owner = uniform(own_w) == vw && l == own_l;
        const bool owner_wave = uniform(own_w) == vw;

        State st;
        if (MODE == 1) {
            const int g0 = Geo::lane_of(vw, vw == 0 ? 0 : Geo::HL);  // first own useful lane
            const int g1 = min(Geo::lane_of(vw, kWave - 1), L.G - 1);
            const int jend = g1 >= g0 ? L.first(g1) + L.count(g1) - 1 : 0;
            st.jbase = g0 < L.G ? L.first(g0) : N + 1;
            const int nown = max(0, jend - st.jbase + 1);
            st.rs = rst + wv * kWave * C;
#pragma unroll
            for (int i = 0; i < C; ++i) {
                const int r = l + kWave * i;
                int gg = 0, kk = 0;
                if (r < nown) L.locate<C>(st.jbase + r - 1, gg, kk);
                st.rd[i] = r < nown ? (gg - Geo::lane_of(vw, 0)) * C + kk : -1;
            }
        }
#pragma unroll
        for (int k = 0; k < C; ++k) st.cur[k] = -INFINITY;  // row 0, columns 1..N
#pragma unroll
        for (int k = 0; k < C; ++k) st.w[k] = 0u;
        st.acc = 0.0;
        st.col0 = col0_value(0, 0.0, T, N);
        st.t = 0;
        const int inf_from = T + 1 - N;  // rows >= inf_from have column 0 = +inf

        if (!H && nch > 0) stage_rows<VS, W>(E, V, 0, min(kChunk, T), lds, x4, cm);
        // SP: halo granules prefetched two chunks ahead, odd chunks in xodd, even in xeven.
        // The chunk loop is unrolled by two for split launches so that each set stays in its
        // own registers (a loop-carried swap would make hipcc wait for both loads).
        uint64_t xodd[C], xeven[C];
        bool xlost = false;  // SP: a hand-off timed out
#pragma unroll
        for (int k = 0; k < C; ++k) xodd[k] = xeven[k] = 0;
        // Prefetches are issued by every lane, unconditionally (chunk and lane clamped into the
        // segment's granule block): a lane- or chunk-conditional load merges into the old
        // value's register, and hipcc then waits for the load right where it is issued.
        const int xl = min(l, Geo::HL - 1) * C;
        if (SP && xsub && !kReg) {
#pragma unroll
            for (int k = 0; k < C; ++k) {
                xodd[k] = granule_load(sp->xin + (int64_t)min(1, nch - 1) * sp->xstride + xl + k);
                xeven[k] = granule_load(sp->xin + (int64_t)min(2, nch - 1) * sp->xstride + xl + k);
            }
        }
#ifdef WX_PHASE_TIMING
        unsigned long long acc_steps = 0, acc_bar = 0, acc_other = 0, x_miss = 0, x_wait = 0, x_slack = 0;
#endif
        // SP: a chunk's bitmap words are stored one chunk late, after the next hand-off wait:
        // that wait drains vmcnt, and a store issued just before it would be waited for too.
        unsigned wdef[C];
#pragma unroll
        for (int k = 0; k < C; ++k) wdef[k] = 0u;
        auto store_deferred = [&](const int qd) {
#pragma unroll
            for (int k = 0; k < C; ++k) st_pub<kWT>(bits + ((int64_t)qd * C + k) * lanes + g, wdef[k]);
        };
        // kReg: the operands of the chunk being computed (o) and of the next one (n), swapped
        // by the two-way unrolled chunk loop
        RegOps opsA, opsB;
        const int etq = (vw == 0 && l == 0) ? VS * 16 : toff[0] * 4;  // quad byte offset of this lane's column
        const int ebq = boff * 4;                                      // ... of the blank (uniform)
        if (kReg) __syncthreads();  // barrier -1 (helper_reg: the column-0 helper's first two chunks)
        // OWN (compile time): the wave holding column N (the only one with column-N stores; the
        // others have no branch around them: a taken branch per eight steps cost the DP waves
        // ~20% of their step time).
        auto chunk_iter = [&](const int q, uint64_t(&xpre)[C], RegOps& o, RegOps& n, auto own) {
            constexpr bool OWN = decltype(own)::value;
            WX_T(c0);
            float* buf = lds + (q % kBufs) * kBufFloats;
            const int rows = min(kChunk, T - q * kChunk);
            float* xq = xh + (q & 1) * W * kWave;
            if (W > 1 && q > 0 && wv < W - 1 && l >= kWave - Geo::HL) {  // publish this chunk's halo
#pragma unroll
                for (int k = 0; k < C; ++k) xq[wv * kWave + (l - (kWave - Geo::HL)) * C + k] = st.cur[k];
            }
            if (SP && xpub && q > 0 && l >= kWave - Geo::HL) {  // ... and to the next part (row 32q)
                uint64_t* go = sp->xout + (int64_t)q * sp->xstride + (l - (kWave - Geo::HL)) * C;
#pragma unroll
                for (int k = 0; k < C; ++k) granule_store(go + k, st.cur[k], sp->tag);
            }
            if (SP && xpub) WX_CQ(q, 1);
            WX_T(c1);
            // this wave's staging (with a helper, DP waves stage nothing).  Single-CU fused
            // launches: not the previous chunk's C bitmap stores, issued last (the wait would
            // expose a store round trip per chunk)
            if (!H) wait_vm();
            __syncthreads();
            WX_T(c2);
            if (wv == 0) WX_CQ(q, 0);
            if (W > 1 && q > 0 && halo && wv > 0) {
#pragma unroll
                for (int k = 0; k < C; ++k) st.cur[k] = xq[(wv - 1) * kWave + l * C + k];
            }
            if (kReg && SP && xsub && q > 0) {  // (the poller's values: Split::xg)
                if (l < Geo::HL) st.cur[0] = sp->xg[(q & 1) * 32 + l];
            } else if (SP && xsub && q > 0) {
                // Halo of row 32q from the previous part: the granules prefetched two chunks
                // ago (the sc1 load takes longer than a chunk).  A part must trail its
                // predecessor by more than the prefetch distance plus the hand-off latency for
                // the prefetch to find them; at chunk 1, and after any miss, it therefore also
                // waits until chunk q + kXSlack is visible (re-building that slack once instead
                // of paying a round trip every chunk).  Waits are bounded: a lost hand-off
                // marks the segment failed.  (An LDS-DMA landing ring with hand-counted vmcnt
                // measured no better.)
                WX_T(x0);
                const bool missed = !xwait(sp->xin, sp->xstride, q, l, sp->tag, xpre, xlost, sp->spin);
                WX_CQ(q, 2);
                if (l < Geo::HL) {
#pragma unroll
                    for (int k = 0; k < C; ++k) st.cur[k] = __builtin_bit_cast(float, (unsigned)xpre[k]);
                }
                WX_T(x1);
                if ((missed || q == 1) && q + kXSlack < nch) {
                    uint64_t tmp[C];
#pragma unroll
                    for (int k = 0; k < C; ++k) tmp[k] = 0;
                    xwait(sp->xin, sp->xstride, q + kXSlack, l, sp->tag, tmp, xlost, sp->spin);
                }
#ifdef WX_PHASE_TIMING
                WX_T(x2);
                x_miss += missed ? 1 : 0;
                x_wait += x1 - x0;
                x_slack += x2 - x1;
#endif
                // this set's next chunk, q + 2 (the old values are dead: keep the load below)
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < C; ++k)
                    xpre[k] = granule_load(sp->xin + (int64_t)min(q + 2, nch - 1) * sp->xstride + xl + k);
            }
            if (SP && MODE == 0 && q > 0 && !halo && g < L.G) store_deferred(q - 1);
            if constexpr (MODE == 2) {
                // checkpoint row 32q (before the chunk's steps; after the barrier, so that the
                // next chunk's vmcnt wait finds these stores a chunk old): the owner lanes' cells
                // in the bitmap word layout, and the fp64 cumsum behind column 0 (wave 0: every
                // lane holds it, alignment.py:368)
                if (!halo && g < L.G) {
                    float* ck = reinterpret_cast<float*>(bits);
#pragma unroll
                    for (int k = 0; k < C; ++k) ck[((int64_t)q * C + k) * lanes + g] = st.cur[k];
                }
                if (!kC0Lds && vw == 0 && l == 0) c0acc[q] = st.acc;
            }
            if (c0prod && q + 1 < nch) c0e = c0_load(q + 1);  // (consumed after this chunk's steps)
            if (!H) {
                if (q + 1 < nch)
                    stage_rows<VS, W>(E, V, (q + 1) * kChunk, min(kChunk, T - (q + 1) * kChunk),
                                      lds + ((q + 1) % kBufs) * kBufFloats, x4, cm);
                if (MODE != 1 && wv == 0 && l < rows) q0[q * kChunk + l] = exp_cr(buf[l * VS]);  // never idle
            }
            const char* bb = reinterpret_cast<const char*>(buf);
            const float* c0q = kC0Lds ? c0b + (q & 1) * kChunk : nullptr;
            WX_T(c3);
            if constexpr (kReg) {
                if (q == 0) reg_load(o, bb, etq, ebq);
                // the next chunk's operands (the last chunk re-reads its own rows: harmless)
                const char* nb = reinterpret_cast<const char*>(lds + ((q + 1 < nch ? q + 1 : q) % kBufs) * kBufFloats);
                float cur0 = st.cur[0];
                reg_chunk<OWN>(o, n, nb, etq, ebq, cur0, st.w[0], owner, cn, q * kChunk, T);
                // Invariant: on a partial last chunk reg_chunk runs all 32 steps on stale rows,
                // so st.cur then holds the cell 32 steps on, not `rows` steps: nothing reads the
                // state after the last chunk (its bits are masked below, column N stops at T).
                // A change that publishes or reads the final cell state must keep
                // hist[(rows - 1) & 7] instead.
                st.cur[0] = cur0;
                st.t += rows;
            } else {
                (void)OWN;
                if (vw == 0) {
                    chunk<true>(bb, c0q, rows, toff, boff, st, inf_from, is_short, halo, f, cnt, owner, N, cn, tr);
                } else {
                    chunk<false>(bb, c0q, rows, toff, boff, st, inf_from, is_short, halo, f, cnt, owner, N, cn, tr);
                }
            }
            if (c0prod && q + 1 < nch) c0_make(q + 1, c0e);  // (read after barrier q + 1)
            WX_T(c4);
#ifdef WX_PHASE_TIMING
            acc_steps += c4 - c3;
            acc_bar += c2 - c1;
            acc_other += (c1 - c0) + (c3 - c2);
#endif
            if (MODE == 0) {
                const int sh = kChunk - rows;  // keep bit 31 = first step of the block
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    // (kReg runs all 32 steps of a partial chunk: bit 31 is already the first
                    // step, the bits of the steps past T are dropped)
                    const unsigned wq = kReg ? (st.w[k] & (0xFFFFFFFFu << sh))
                                             : ((sh == 0) ? st.w[k] : (st.w[k] << sh));
                    if (SP)
                        wdef[k] = wq;
                    else if (!halo && g < L.G)  // (lanes past column N: words the walk never reads)
                        bits[((int64_t)q * C + k) * lanes + g] = wq;
                    st.w[k] = 0u;
                }
            }
        };
        if constexpr (SP) {
            auto loop = [&](auto own) {
                for (int q = 0; q < nch; q += 2) {
                    chunk_iter(q, xeven, opsA, opsB, own);
                    if (q + 1 < nch) chunk_iter(q + 1, xodd, opsB, opsA, own);
                }
            };
            if (owner_wave)
                loop(BoolTag<true>{});
            else
                loop(BoolTag<false>{});
            if (MODE == 0 && nch > 0 && !halo && g < L.G) store_deferred(nch - 1);
        } else {
            for (int q = 0; q < nch; ++q) chunk_iter(q, xeven, opsA, opsB, BoolTag<true>{});
        }
#ifdef WX_PHASE_TIMING
        if (l == 0 && blockIdx.x < 8192 && MODE != 1) {
            unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + wv) * 3;
            o[0] = acc_steps;
            o[1] = acc_bar;
            o[2] = acc_other;
            if (SP && xsub) {  // hand-off: missed prefetches, cycles in the chunk's wait, in slack waits
                unsigned long long* x = wx_loop + ((size_t)blockIdx.x * kLoopSlots + 14) * 3;
                x[0] = x_miss;
                x[1] = x_wait;
                x[2] = x_slack;
            }
        }
#endif
        return xlost;
    }

    // ---------------------------------------------------------------- register-resident chunks
    struct RegOps {
        float4 et[kChunk / 4];  // em[t, tok] of this lane's cell (column-1 wave, lane 0: col0_pre's value)
        float4 eb[kChunk / 4];  // em[t, blank]
    };
    __device__ __forceinline__ static void reg_load(RegOps& o, const char* buf, int etq, int ebq) {
#pragma unroll
        for (int p = 0; p < kChunk / 4; ++p) {
            o.et[p] = *reinterpret_cast<const float4*>(buf + p * kQS * 4 + etq);
            o.eb[p] = *reinterpret_cast<const float4*>(buf + p * kQS * 4 + ebq);
        }
    }
    __device__ __forceinline__ static float comp(const float4& v, int j) {
        return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
    }
    // Four time steps of one cell (alignment.py:372-378), hand-ordered so that the chain
    // through the cell value (maximum -> next step's DPP add) needs no wait states: the DPP's
    // source is read two instructions after the maximum that wrote it (the addc and the stay
    // add sit in between).  One asm block per four steps: hipcc cannot see inside a block and
    // pads an s_nop at every block boundary whose next block might read a fresh VGPR through
    // DPP.  Lane 0's left input is zero-filled: in the column-1 wave its operand `et` is
    // col0_pre's tr[t][0] + em[t, tok[0]] (0 + x is x for every x the DP can tell apart: it
    // only compares values and takes maxima), elsewhere a halo lane's don't-care.  n[k] =
    // the cell value after step k.
#define WX_REG_STEP(CUR, NC, ET, EB)                                                                  \
    "v_add_f32 %[s], %[" #CUR "], %[" #EB "]\n\t"                                                   \
    "v_add_f32_dpp %[c], %[" #CUR "], %[" #ET "] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
    "v_cmp_gt_f32 vcc, %[c], %[s]\n\t"                                                              \
    "v_maximum3_f32 %[" #NC "], %[s], %[c], %[c]\n\t"                                               \
    "v_addc_co_u32 %[w], vcc, %[w], %[w], vcc\n\t"
#define WX_REG_OPERANDS                                                                                 \
    : [n0] "=&v"(n[0]), [n1] "=&v"(n[1]), [n2] "=&v"(n[2]), [n3] "=&v"(n[3]), [w] "+v"(w), [s] "=&v"(s),  \
      [c] "=&v"(c)                                                                                          \
    : [cur] "v"(cur), [e0] "v"(et.x), [e1] "v"(et.y), [e2] "v"(et.z), [e3] "v"(et.w), [b0] "v"(eb.x),     \
      [b1] "v"(eb.y), [b2] "v"(eb.z), [b3] "v"(eb.w)                                                         \
    : "vcc"
    template <bool FIRST>  // FIRST: `cur` may have just been written by a VALU op (halo copy-in)
    __device__ __forceinline__ static void reg_steps4(float cur, unsigned& w, const float4& et, const float4& eb,
                                                      float (&n)[4]) {
        float s, c;
        if constexpr (FIRST)
            asm volatile("s_nop 1\n\t" WX_REG_STEP(cur, n0, e0, b0) WX_REG_STEP(n0, n1, e1, b1)
                             WX_REG_STEP(n1, n2, e2, b2) WX_REG_STEP(n2, n3, e3, b3) WX_REG_OPERANDS);
        else
            asm volatile(WX_REG_STEP(cur, n0, e0, b0) WX_REG_STEP(n0, n1, e1, b1) WX_REG_STEP(n1, n2, e2, b2)
                             WX_REG_STEP(n2, n3, e3, b3) WX_REG_OPERANDS);
    }
#undef WX_REG_OPERANDS
#undef WX_REG_STEP
    // 32 steps on operands `o`, issuing the next chunk's operand reads (n, from buffer nb) one
    // quad ahead of each group of four steps; column N history stored by the owner lane (rows
    // past T skipped: the steps of a partial chunk past T compute on stale rows, harmlessly).
    // OWN: this wave holds column N (the others have no column-N code)
    template <bool OWN>
    __device__ __forceinline__ static void reg_chunk(const RegOps& o, RegOps& n, const char* nb, int etq, int ebq,
                                                     float& cur, unsigned& w, bool owner, float* __restrict__ cn,
                                                     int t0, int T) {
        float hist[OWN ? kChunk : 1];
#pragma unroll
        for (int p = 0; p < kChunk / 4; ++p) {
            n.et[p] = *reinterpret_cast<const float4*>(nb + p * kQS * 4 + etq);
            n.eb[p] = *reinterpret_cast<const float4*>(nb + p * kQS * 4 + ebq);
            __builtin_amdgcn_sched_barrier(0);
            float nv[4];
            if (p == 0)
                reg_steps4<true>(cur, w, o.et[p], o.eb[p], nv);
            else
                reg_steps4<false>(cur, w, o.et[p], o.eb[p], nv);
            if constexpr (OWN) {
#pragma unroll
                for (int j = 0; j < 4; ++j) hist[4 * p + j] = nv[j];
            }
            cur = nv[3];
            __builtin_amdgcn_sched_barrier(0);
        }
        if (OWN && owner) {
            // rows t0 + 1 .. t0 + 32 -> cn[t0 .. t0 + 31], once per chunk and whole: rows past T
            // land in the segment's padding (kCnPad).  (Stored per 8 steps inside the chain,
            // with a partial-group path, they cost the pacing wave a taken branch and an EXEC
            // round trip per 8 steps: 59.7 -> 55.3 -> ... us.)
            // Eight 16-byte stores, written through (sc1, kWT): the last part reads them with
            // sc1 loads and the arrival needs no release (32 single 4-byte sc1 stores had cost
            // more than the release).
#pragma unroll
            for (int i = 0; i < kChunk / 4; ++i)
                st_pub4<kWT>(cn, t0 + 4 * i, make_float4(hist[4 * i], hist[4 * i + 1], hist[4 * i + 2], hist[4 * i + 3]));
        }
    }
    // tr[t][0] + em[t, tok[0]] for the rows of chunk q (the column-1 wave's lane-0 operand),
    // into column VS of the chunk's quad buffer.  tr[t][0] (alignment.py:367-370): 0 at t = 0,
    // fp32 of the fp64 sum of em[0..t-1, 0] (torch CPU cumsum accumulates in double, in row
    // order), +inf in the last N rows.  The sums: col0_chunk.
    __device__ __forceinline__ static void col0_pre(int q, const SegDesc& d, float* buf, int tok0, double& acc) {
        const int T = d.T, N = d.N;
        const int l = lane_id();
        const int rr = l & 31;
        // both operands of the row read up front: one LDS round trip instead of two
        const float e = buf[(rr >> 2) * kQS + (rr & 3)];              // em[t, 0]
        const float et = buf[(rr >> 2) * kQS + 4 * tok0 + (rr & 3)];  // em[t, tok[0]]
        const double a = col0_chunk(acc, e);
        if (l < 32) {
            const int t = q * kChunk + l;
            buf[(l >> 2) * kQS + 4 * VS + (l & 3)] = col0_value(t, a, T, N) + et;
        }
    }
    // Staging of the quad layout.  Rows are first copied row-major into a ring of kRing raw
    // chunk buffers by 16-byte LDS-DMA (stage_rows: 4 instructions per chunk when V == 32,
    // issued kRing - 1 chunks ahead, so each chunk has two chunk-times to land), then
    // transposed LDS -> LDS into the quad buffer: lane i reads the 4 rows of its (row quad,
    // column) pairs (two ds_read2_b32) and writes them as one 16-byte store.  (One-dword LDS-DMA
    // straight into the quad layout needs 16 instructions per chunk: measured ~1,600 cycles of
    // issue per chunk, more than a DP chunk; register staging one chunk ahead stalled on the
    // loads.)
    static constexpr int kRing = 4;  // (A/B: 8 was 1.5 us slower on config 2)
    static constexpr int kPairs = 8 * VS / kWave;  // (row quad, column) pairs per lane
    __device__ __forceinline__ static void transpose_quads(const float* raw, float* buf) {
        const int l = lane_id();
        float v[kPairs][4];
#pragma unroll
        for (int m = 0; m < kPairs; ++m) {
            const int k = kWave * m + l, p = k / VS, col = k % VS;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[m][j] = raw[(4 * p + j) * VS + col];
        }
#pragma unroll
        for (int m = 0; m < kPairs; ++m) {
            const int k = kWave * m + l, p = k / VS, col = k % VS;
            *reinterpret_cast<float4*>(buf + p * kQS + 4 * col) = make_float4(v[m][0], v[m][1], v[m][2], v[m][3]);
        }
    }
    // The two helpers of a register-resident split kernel.  Barriers: -1, then one per chunk.
    // Wave W (the stager) makes chunk q + 2's quad buffer ready before barrier q (transposed
    // out of the raw ring, its DMA issued two iterations earlier); wave W + 1 (part 0 only)
    // writes col0_pre of chunks 0 and 1 after barrier -1 and of chunk q + 2 after barrier q.
    // So after barrier q the DP waves can read chunk q + 1's operands, col0_pre included,
    // while they compute chunk q.  Quad buffer (q + 2) % kBufs (five) last held chunk q - 3,
    // whose operand reads the DP waves waited for before chunk q - 3's steps and whose column
    // 0 the helper read during chunk q - 5.
    // The stager of a V == 32 batch with 16-byte aligned rows, through registers: lane l loads
    // 16 bytes (columns 4 cg .. 4 cg + 3, cg = (l >> 2) & 7) of row 8 i + 4 h + j (j = l & 3,
    // h = l >> 5) of a chunk with one global_load_dwordx4 per i (4 per chunk) and writes them
    // into the quad layout with 16 ds_write_b32 (row quad 2 i + h, columns 4 cg + m, row j):
    // no LDS-DMA ring and no LDS -> LDS transpose (which cost ~1,200 cycles per chunk and paced
    // every part).  Four register sets: chunk c is loaded at iteration c - 6 (rows clamped into
    // the segment, so the loads are unconditional and the compiler counts them exactly) and
    // written before barrier c - 2, so each load has four chunk-times to land.
    static constexpr int kStgSets = 4;
    struct StgSet {
        float4 v[4];
    };
    __device__ __forceinline__ static void stg_load(StgSet& s, const float* __restrict__ E, int T, int c) {
        const int l = lane_id();
        const int r = 4 * (l >> 5) + (l & 3), cg = (l >> 2) & 7;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = min(c * kChunk + 8 * i + r, T - 1);
            s.v[i] = *reinterpret_cast<const float4*>(E + (int64_t)t * 32 + 4 * cg);
        }
    }
    __device__ __forceinline__ static void stg_write(const StgSet& s, float* buf) {
        const int l = lane_id();
        const int cg = (l >> 2) & 7;
        float* o = buf + (l >> 5) * kQS + 16 * cg + (l & 3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i * kQS + 0] = s.v[i].x;
            o[2 * i * kQS + 4] = s.v[i].y;
            o[2 * i * kQS + 8] = s.v[i].z;
            o[2 * i * kQS + 12] = s.v[i].w;
        }
    }
    __device__ static void stager_regs(const SegDesc& d, const float* __restrict__ E, float* lds, int nch) {
        static_assert(VS == 32, "register staging is for 32-float rows");
        const int T = d.T;
        auto buf = [&](int q) { return lds + (q % kBufs) * kBufFloats; };
        StgSet s0, s1, s2, s3;
        stg_load(s0, E, T, 0);
        stg_load(s1, E, T, 1);
        stg_load(s2, E, T, 2);
        stg_load(s3, E, T, 3);
        stg_write(s0, buf(0));
        stg_write(s1, buf(1));
        stg_load(s0, E, T, 4);
        stg_load(s1, E, T, 5);
        __syncthreads();  // barrier -1
        // iteration q: chunk q + 2 (set (q + 2) % 4) into its quad buffer, then chunk q + 6 into
        // that set; barrier q
        auto iter = [&](int q, StgSet& s) {
            if (q + 2 < nch) stg_write(s, buf(q + 2));
            stg_load(s, E, T, q + 6);
            __syncthreads();  // barrier q
        };
        int q = 0;
        for (; q + 4 <= nch; q += 4) {
            iter(q, s2);
            iter(q + 1, s3);
            iter(q + 2, s0);
            iter(q + 3, s1);
        }
        if (q < nch) iter(q++, s2);
        if (q < nch) iter(q++, s3);
        if (q < nch) iter(q++, s0);
        wait_vm();  // (no load outlives the wave)
    }

    // The idle helper of a part > 0 (register-resident kernels): chunk q's halo granules from
    // part p - 1 into Split::xg[q & 1], re-reading until every tag matches (bounded: returns
    // whether the hand-off was lost).  Only loads in this wave.  `pre` holds chunk q's first
    // read, issued before barrier q - 1 (so a part that trails its predecessor finds the
    // granules without a round trip inside its chunk); chunk q + 1's is issued on the way out.
    __device__ static bool poll_halo(const Split* sp, int q, int nch, bool lost, uint64_t& pre) {
        constexpr int HL = Geo::HL;
        const int l = lane_id();
        const uint64_t* gi = sp->xin + (int64_t)q * sp->xstride + min(l, HL - 1) * C;
        uint64_t x = pre;
        bool ok = l >= HL || (unsigned)(x >> 32) == sp->tag;
        for (int it = 0; !lost && !__all(ok) && it < sp->spin; ++it) {
            x = granule_load(gi);
            ok = l >= HL || (unsigned)(x >> 32) == sp->tag;
        }
        if (l < HL) sp->xg[(q & 1) * 32 + l] = __builtin_bit_cast(float, (unsigned)x);
        pre = granule_load(gi + (int64_t)(min(q + 1, nch - 1) - q) * sp->xstride);
        return !__all(ok);
    }
    __device__ static bool helper_reg(const SegDesc& d, const float* __restrict__ E, int V, float* lds, float* raw,
                                      int nch, int tok0, bool col0, bool stage, bool x4, const Split* sp = nullptr) {
        const int T = d.T;
        // the idle helper of a part > 0 that holds columns (the previous part publishes nothing
        // for a part without any)
        const bool poll = SP && !col0 && !stage && sp && sp->p > 0 &&
                          Geo::lane_of(sp->p * W, Geo::HL) < Layout::make(C, d.N, sp->lanes).G;
        bool lost = false;
        if constexpr (VS == 32) {
            if (stage && x4 && !col0) {
                stager_regs(d, E, lds, nch);
                return false;
            }
        }
        auto buf = [&](int q) { return lds + (q % kBufs) * kBufFloats; };
        auto ring = [&](int q) { return raw + (q % kRing) * kChunk * VS; };
        auto rows_of = [&](int q) { return (q >= 0 && q < nch) ? min(kChunk, T - q * kChunk) : 0; };
        const ColMap cm{};  // (VS != kGatherVS: unused)
        auto issue = [&](int q) {
            if (q < nch) stage_rows<VS, 1, true>(E, V, q * kChunk, rows_of(q), ring(q), x4, cm);
        };
        // waits by DMA instruction count (stage_rows: one 16-byte instruction per 8 rows, else one
        // per row); the loads complete in order, so "at most n in flight" = everything but the
        // newest n landed
        auto instrs = [&](int q) { return q < nch ? (x4 && VS == 32 ? (rows_of(q) + 7) / 8 : rows_of(q)) : 0; };
        auto wait_all_but = [&](int q0, int q1) {  // all but chunks [q0, q1)'s DMA instructions landed
            int n = 0;
            for (int c = q0; c < q1; ++c) n += instrs(c);
            if (n >= 60) asm volatile("s_waitcnt vmcnt(60)" ::: "memory");
            else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
            else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
            else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        if (stage) {
            for (int q = 0; q < kRing - 1; ++q) issue(q);
            wait_all_but(2, kRing - 1);  // chunks 0 and 1 landed
            transpose_quads(ring(0), buf(0));
            if (nch > 1) transpose_quads(ring(1), buf(1));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot 0's reads done before its reuse
            issue(kRing - 1);
        }
        double acc = 0.0;
        uint64_t pre = 0;  // poll: chunk 1's granules (first read)
        if (poll) pre = granule_load(sp->xin + (int64_t)min(1, nch - 1) * sp->xstride + min(lane_id(), Geo::HL - 1) * C);
        __syncthreads();  // barrier -1
        if (col0) {
            col0_pre(0, d, buf(0), tok0, acc);
            if (nch > 1) col0_pre(1, d, buf(1), tok0, acc);
        }
#ifdef WX_PHASE_TIMING
        unsigned long long acc_work = 0, acc_bar = 0, acc_vm = 0;
#endif
        // one iteration: stage (chunk q + 2 transposed out of the ring — issued two iterations ago;
        // chunk q + 3's DMA may still be in flight — then chunk q + kRing issued into the slot of
        // chunk q, transposed two iterations ago), barrier q, column 0
        for (int q = 0; q < nch; ++q) {
            WX_T(h0);
#ifdef WX_PHASE_TIMING
            unsigned long long hw = h0;
#endif
            if (stage && q + 2 < nch) {
                wait_all_but(q + 3, q + kRing);  // chunk q + 2's DMA landed (later ones may be in flight)
#ifdef WX_PHASE_TIMING
                hw = __builtin_amdgcn_s_memtime();
#endif
                transpose_quads(ring(q + 2), buf(q + 2));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // its reads done: the slot is free
                issue(q + kRing);
            }
            if (poll && q > 0) {
                lost = poll_halo(sp, q, nch, lost, pre) || lost;
#ifdef WX_PHASE_TIMING
                hw = __builtin_amdgcn_s_memtime();  // (the poll counts as the DMA wait)
#endif
            }
            WX_T(h1);
            __syncthreads();  // barrier q
            WX_T(h2);
            if (col0 && q + 2 < nch) col0_pre(q + 2, d, buf(q + 2), tok0, acc);
            WX_T(h3);
#ifdef WX_PHASE_TIMING
            acc_vm += hw - h0;
            acc_bar += h2 - h1;
            acc_work += (h3 - h2) + (h1 - hw);
#endif
        }
#ifdef WX_PHASE_TIMING
        if (lane_id() == 0 && blockIdx.x < 8192) {  // [work, barrier wait, DMA wait] per helper
            unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + W + (stage ? 0 : 1)) * 3;
            o[0] = acc_work;
            o[1] = acc_bar;
            o[2] = acc_vm;
        }
#endif
        return lost;
    }

    // The helper wave (H): mirrors the DP waves' barriers.  Before barrier q, chunks q and
    // q+1 are staged and column 0 of chunk q is in c0b[q & 1].  (q0 is filled after the
    // forward pass, while wave 0 walks: fill_q0.)
    __device__ static void helper(const SegDesc& d, const float* __restrict__ E, int V, float* lds, float* c0b,
                                  int nch, bool x4, const ColMap& cm, bool col0, bool stage = true) {
        const int T = d.T, N = d.N;
        const int inf_from = T + 1 - N;
        double acc = 0.0;  // sum of em[0..t-1, 0], uniform
        // Rows are staged three chunks ahead (four LDS buffers) and waited for one chunk
        // ahead, so each chunk's loads have two chunk times to land: at chunk q only the
        // loads of chunk q+2 may still be in flight (vmcnt = that chunk's instruction
        // count: 4 for 16-byte staging, 32 for row staging; gathers drain fully).
        if (stage) {
            for (int i = 0; i < 3 && i < nch; ++i)
                stage_rows<VS, 1, true>(E, V, i * kChunk, min(kChunk, T - i * kChunk), lds + i * kBufFloats, x4, cm);
            wait_vm();
        }
        // chunk 0's column 0: from the staged rows, or (a column-only helper, which cannot
        // know when the other helper's staging landed) straight from the emission rows
        if (col0) {
            if (stage) {
                column0(0, T, inf_from, lds, c0b, acc);
            } else {  // chunk 0 column 0 into the 4th buffer (first staged after barrier 0)
                float* own = lds + 3 * kBufFloats;
                if (lane_id() < min(kChunk, T)) own[lane_id() * VS] = E[(int64_t)lane_id() * V];
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                column0(0, T, inf_from, own, c0b, acc);
            }
        }
#ifdef WX_PHASE_TIMING
        unsigned long long acc_c0 = 0, acc_bar = 0, acc_other = 0;
#endif
        for (int q = 0; q < nch; ++q) {
            WX_T(h0);
            // chunk q+1 must have landed; chunk q+2 (staged at q-1) may still be in flight
            if (!stage) {
            } else if (q + 2 < nch && T - (q + 2) * kChunk >= kChunk && VS != kGatherVS) {
                if (x4 && VS == 32)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            } else {
                wait_vm();
            }
            WX_T(h1);
            __syncthreads();
            WX_T(h2);
            if (stage && q + 3 < nch)
                stage_rows<VS, 1, true>(E, V, (q + 3) * kChunk, min(kChunk, T - (q + 3) * kChunk),
                                        lds + ((q + 3) % kBufs) * kBufFloats, x4, cm);
            WX_T(h3);
            if (col0 && q + 1 < nch)
                column0(q + 1, T, inf_from, lds + ((q + 1) % kBufs) * kBufFloats, c0b, acc);
            WX_T(h4);
#ifdef WX_PHASE_TIMING
            acc_c0 += h4 - h3;
            acc_bar += h2 - h1;
            acc_other += (h1 - h0) + (h3 - h2);
#endif
        }
#ifdef WX_PHASE_TIMING
        if (lane_id() == 0 && blockIdx.x < 8192) {
            unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + W + (stage ? 0 : 1)) * 3;
            o[0] = acc_c0;
            o[1] = acc_bar;
            o[2] = acc_other;
        }
#endif
    }

    // Column 0 of chunk q (tr[t][0], alignment.py:367-370: 0, fp32(fp64 cumsum), +inf in
    // the last N rows) into c0b[q & 1][r].  The fp64 chain runs on wave-uniform values (rows
    // read as LDS broadcasts, converted ahead), one dependent v_add_f64 per row; rows past
    // the segment's end feed only values nobody reads.
    __device__ __forceinline__ static void column0(int q, int T, int inf_from, const float* buf, float* c0b,
                                                   double& acc) {
        const int t0 = q * kChunk;
        float* out = c0b + (q & 1) * kChunk;
        float e[kChunk];
#pragma unroll
        for (int r = 0; r < kChunk; ++r) e[r] = buf[r * VS];  // uniform address: broadcast
#pragma unroll
        for (int r = 0; r < kChunk; ++r) {
            out[r] = (float)acc;  // tr[t0 + r][0] before the +inf / row-0 fix-up
            acc += (double)e[r];
        }
        const int l = lane_id();
        if (l < kChunk) {
            const int t = t0 + l;
            const float v = out[l];
            out[l] = (t >= inf_from) ? INFINITY : (t == 0 ? 0.0f : v);
        }
    }

    // One chunk's steps: unrolled groups of kUnroll with immediate LDS row offsets, then the
    // remainder.  WAVE0: this wave holds column 1 (its left input is column 0).
    template <bool WAVE0>
    __device__ __forceinline__ static void chunk(const char* bb, const float* c0q, int rows, const int (&toff)[C],
                                                 int boff, State& st, int inf_from, bool is_short, bool halo, int f,
                                                 int cnt, bool owner, int N, float* __restrict__ cn,
                                                 float* __restrict__ tr) {
        constexpr int kColLds = 3, kColFinite = 1, kColAny = 2;
        if (kPipelined && rows == kChunk) {  // software-pipelined full chunk
            if (!WAVE0)
                pipelined_chunk<0>(bb, c0q, toff, boff, st, inf_from, false, halo, f, cnt, owner, N, cn, tr);
            else if (kC0Lds)
                pipelined_chunk<kColLds>(bb, c0q, toff, boff, st, inf_from, is_short, halo, f, cnt, owner, N, cn, tr);
            else if (st.t + kChunk < inf_from)
                pipelined_chunk<kColFinite>(bb, c0q, toff, boff, st, inf_from, is_short, halo, f, cnt, owner, N, cn, tr);
            else
                pipelined_chunk<kColAny>(bb, c0q, toff, boff, st, inf_from, is_short, halo, f, cnt, owner, N, cn, tr);
            return;
        }
        int r = 0;
        for (; r + kU <= rows; r += kU) {
            const char* gb = bb + r * kRowBytes;
            const char* ga[C];
#pragma unroll
            for (int k = 0; k < C; ++k) ga[k] = gb + toff[k];
            float hist[kU];  // column N after each step (owner lane)
            if (!WAVE0 || kC0Lds || st.t + kU < inf_from) {  // column 0 from LDS, or finite for the group
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    step<!WAVE0 ? 0 : (kC0Lds ? kColLds : kColFinite)>(gb, ga, u * kRowBytes, boff, c0q + r + u, st,
                                                                 inf_from, is_short, halo, f, cnt, N, tr);
                    hist[u] = st.cur[C - 1];
                    ++st.t;
                }
            } else {
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    step<kColAny>(gb, ga, u * kRowBytes, boff, c0q, st, inf_from, is_short, halo, f, cnt, N, tr);
                    hist[u] = st.cur[C - 1];
                    ++st.t;
                }
            }
            if (MODE != 1 && owner) {  // rows t-kU+1 .. t at cn[t-kU .. t-1] (16-byte aligned)
#pragma unroll
                for (int i = 0; i < kU / 4; ++i)
                    st_pub4<kWT>(cn, st.t - kU + 4 * i, make_float4(hist[4 * i], hist[4 * i + 1], hist[4 * i + 2], hist[4 * i + 3]));
            }
        }
        for (; r < rows; ++r) {
            const char* gb = bb + r * kRowBytes;
            const char* ga[C];
#pragma unroll
            for (int k = 0; k < C; ++k) ga[k] = gb + toff[k];
            step<!WAVE0 ? 0 : (kC0Lds ? kColLds : kColAny)>(gb, ga, 0, boff, c0q + r, st, inf_from, is_short, halo, f,
                                                       cnt, N, tr);
            if (MODE != 1 && owner) st_pub<kWT>(cn + st.t, st.cur[C - 1]);
            ++st.t;
        }
    }

    // A full 32-step chunk with the LDS operands of step u+2 and u+3 loaded while step u
    // computes.  sched_barrier keeps the scheduler from sinking the loads back to their uses
    // (it does, to minimise registers); the waitcnt pass counts them exactly, since LDS
    // returns in order.
    template <int COL>
    __device__ __forceinline__ static void pipelined_chunk(const char* bb, const float* c0q, const int (&toff)[C],
                                                           int boff, State& st, int inf_from, bool is_short,
                                                           bool halo, int f, int cnt, bool owner, int N,
                                                           float* __restrict__ cn, float* __restrict__ tr) {
        const char* ga[C];
#pragma unroll
        for (int k = 0; k < C; ++k) ga[k] = bb + toff[k];
        Row rw[kChunk];
        // COL 3 (column 0 from the helper's LDS row): the chunk's 32 values in 8 16-byte
        // loads up front instead of an address move + ds_read_b32 per step in the wave that
        // paces the chain (the column-1 wave)
        float c0r[COL == 3 ? kChunk : 1];
        if constexpr (COL == 3) {
#pragma unroll
            for (int i = 0; i < kChunk / 4; ++i) {
                const float4 v = reinterpret_cast<const float4*>(c0q)[i];
                c0r[4 * i] = v.x;
                c0r[4 * i + 1] = v.y;
                c0r[4 * i + 2] = v.z;
                c0r[4 * i + 3] = v.w;
            }
        }
        constexpr int LC = COL == 3 ? 4 : COL;  // load_row without the per-step column-0 read
        auto c0_of = [&](Row& r, int u) {
            if constexpr (COL == 3) r.c0 = c0r[u];
        };
        load_row<LC>(bb, ga, 0, boff, c0q, rw[0]);
        load_row<LC>(bb, ga, kRowBytes, boff, c0q + 1, rw[1]);
        c0_of(rw[0], 0);
        c0_of(rw[1], 1);
        float hist[kUnroll];
#pragma unroll
        for (int u = 0; u < kChunk; ++u) {
            if ((u & 1) == 0 && u + 2 < kChunk) {
                load_row<LC>(bb, ga, (u + 2) * kRowBytes, boff, c0q + u + 2, rw[u + 2]);
                load_row<LC>(bb, ga, (u + 3) * kRowBytes, boff, c0q + u + 3, rw[u + 3]);
                c0_of(rw[u + 2], u + 2);
                c0_of(rw[u + 3], u + 3);
            }
            __builtin_amdgcn_sched_barrier(0);
            advance<COL>(bb, u * kRowBytes, c0q + u, rw[u], st, inf_from, is_short, halo, f, cnt, N, tr);
            hist[u & (kUnroll - 1)] = st.cur[C - 1];
            ++st.t;
            if (MODE != 1 && (u & (kUnroll - 1)) == kUnroll - 1 && owner) {
                st_pub4<kWT>(cn, st.t - kUnroll, make_float4(hist[0], hist[1], hist[2], hist[3]));
                st_pub4<kWT>(cn, st.t - kUnroll + 4, make_float4(hist[4], hist[5], hist[6], hist[7]));
            }
        }
    }

    // One time step t -> t+1 (alignment.py:372-378).  COL: 0 = not the column-1 wave (lane
    // 0's left input is a halo edge, don't-care); column-1 wave: 1 = column 0 finite for the
    // next row, 2 = general column 0, 3 = column 0 read from the helper's LDS row.
    template <int COL>
    __device__ __forceinline__ static void step(const char* gb, const char* (&ga)[C], int ro, int boff,
                                                const float* c0, State& st, int inf_from, bool is_short, bool halo,
                                                int f, int cnt, int N, float* __restrict__ tr) {
        Row rw;
        load_row<COL>(gb, ga, ro, boff, c0, rw);
        advance<COL>(gb, ro, c0, rw, st, inf_from, is_short, halo, f, cnt, N, tr);
    }

    // The LDS operands of one step: em[t, blank], em[t, tok[j-1]] per slot, column 0 (COL 3).
    struct Row {
        float eb;
        float et[C];
        float c0;
    };
    template <int COL>
    __device__ __forceinline__ static void load_row(const char* gb, const char* (&ga)[C], int ro, int boff,
                                                    const float* c0, Row& rw) {
        rw.eb = *reinterpret_cast<const float*>(gb + ro + boff);
#pragma unroll
        for (int k = 0; k < C; ++k) rw.et[k] = *reinterpret_cast<const float*>(ga[k] + ro);
        if (COL == 3) rw.c0 = *c0;
        if (COL == 1 || COL == 2) rw.c0 = *reinterpret_cast<const float*>(gb + ro);  // em[t, 0]
    }

    template <int COL>
    __device__ __forceinline__ static void advance(const char* gb, int ro, const float* c0, const Row& rw, State& st,
                                                   int inf_from, bool is_short, bool halo, int f, int cnt, int N,
                                                   float* __restrict__ tr) {
        const float eb = rw.eb;
        const float(&et)[C] = rw.et;
        // last cell of the lane to the left (short lanes end at slot C-2)
        const float src = (C > 1 && is_short) ? st.cur[C > 1 ? C - 2 : 0] : st.cur[C - 1];
        // Lane 0's left input is column 0 in the column-1 wave and a halo lane's don't-care
        // elsewhere: there the DPP zero-fills (bound_ctrl).  In the column-1 wave lane 63
        // passes column 0 round to lane 0 instead (wave_ror:1; lane 63's own last cell feeds
        // no lane of this wave).  Either way every lane's source is a plain register, so
        // hipcc fuses the shift into the add (v_add_f32_dpp) and no v_mov sets up `old`.
        float left;
        if (COL) {
            const float c0v = COL == 3 ? rw.c0 : st.col0;
            const float src2 = lane_id() == kWave - 1 ? c0v : src;
            left = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, src2), 0x13C /* wave_ror:1 */,
                                                                      0xF, 0xF, true));  // (no lane is out of range)
        } else {
            left = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, src), 0x138 /* wave_shr:1 */,
                                                                      0xF, 0xF, true));
        }
#pragma unroll
        for (int k = C - 1; k >= 0; --k) {
            const float s = st.cur[k] + eb;
            const float c = (k == 0 ? left : st.cur[k > 0 ? k - 1 : 0]) + et[k];
            if (MODE == 0) st.w[k] = shift_in(st.w[k], c, s);
            st.cur[k] = nan_max(s, c);
        }
        if (COL == 1 || COL == 2) {
            const float e0 = rw.c0;
            st.acc += (double)e0;
            st.col0 = (COL == 1 || st.t + 1 < inf_from) ? (float)st.acc : INFINITY;
        }
        if (MODE == 1) {
            float* row = tr + (int64_t)(st.t + 1) * ((int64_t)N + 1);
            if (COL && lane_id() == 0)
                row[0] = COL == 3 ? (st.t + 1 < inf_from ? c0[1] : INFINITY) : st.col0;
            float* rw = st.rs + lane_id() * C;  // every lane stages its C slots (in-order LDS)
            if constexpr (C % 4 == 0) {
#pragma unroll
                for (int k = 0; k < C; k += 4)
                    *reinterpret_cast<float4*>(rw + k) = make_float4(st.cur[k], st.cur[k + 1], st.cur[k + 2], st.cur[k + 3]);
            } else if constexpr (C % 2 == 0) {
#pragma unroll
                for (int k = 0; k < C; k += 2) *reinterpret_cast<float2*>(rw + k) = make_float2(st.cur[k], st.cur[k + 1]);
            } else {
#pragma unroll
                for (int k = 0; k < C; ++k) rw[k] = st.cur[k];
            }
            float* own = row + st.jbase + lane_id();
#pragma unroll
            for (int i = 0; i < C; ++i)
                if (st.rd[i] >= 0) own[kWave * i] = st.rs[st.rd[i]];  // (nt stores: 25% slower)
        }
    }
};

// q0[t] = exp(em[t, 0]) for rows [0, T), by the threads [first_thread, blockDim) (the waves
// that do not walk).
__device__ void fill_q0(const float* __restrict__ E, int V, int T, float* __restrict__ q0, int first_thread) {
    const int n = (int)blockDim.x - first_thread;
    for (int t = (int)threadIdx.x - first_thread; t < T; t += n) q0[t] = exp_cr(E[(int64_t)t * V]);
}

// Argmax of column N over rows 0..T with torch.argmax semantics (first maximum; the first
// NaN wins), rows 1..T read from cn[0..T-1], row 0 = -inf (alignment.py:395-396).  Wave 0.
template <bool WT = false>  // WT: sc1 loads (a split segment's history, written through by another CU)
__device__ int column_argmax(const float* __restrict__ cn, int T) {
    const int l = lane_id();
    int nan_row = 0x7fffffff, best_row = 0;
    float best = -INFINITY;
    // loads in flight per lane.  WT: the history was written through, so every load goes out
    // to the fabric (~1 us): one round for T <= 2048 (8 per lane took 3 rounds at T = 1499)
    constexpr int kBatch = WT ? 32 : 8;
    for (int base = 0; base < T; base += kBatch * kWave) {
        float v[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {  // (unconditional, clamped: no wait at the issue)
            const int i = base + u * kWave + l;
            v[u] = ld_pub<WT>(cn + min(i, T - 1));
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
            if (base + u * kWave + l >= T) v[u] = -INFINITY;
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {  // rows of a lane in increasing order
            const int row = base + u * kWave + l + 1;
            if (v[u] != v[u]) {
                nan_row = min(nan_row, row);
            } else if (v[u] > best) {
                best = v[u];
                best_row = row;
            }
        }
    }
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        nan_row = min(nan_row, __shfl_xor(nan_row, off));
        const float b2 = __shfl_xor(best, off);
        const int r2 = __shfl_xor(best_row, off);
        if (b2 > best || (b2 == best && r2 < best_row)) {
            best = b2;
            best_row = r2;
        }
    }
    return uniform(nan_row != 0x7fffffff ? nan_row : best_row);
}

// column_argmax with every thread of a multi-wave workgroup (all threads must call it):
// rows strided over the threads, 8 loads in flight each, then a wave reduction and one LDS
// exchange (red: 3 ints per wave).  Same semantics: first maximum, the first NaN wins.
__device__ int block_argmax(const float* __restrict__ cn, int T, int* red) {
    const int tid = (int)threadIdx.x, n = (int)blockDim.x;
    int nan_row = 0x7fffffff, best_row = 0;
    float best = -INFINITY;
    constexpr int kBatch = 8;
    for (int base = tid; base < T; base += kBatch * n) {
        float v[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            const int i = base + u * n;
            v[u] = i < T ? cn[i] : -INFINITY;
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {  // this thread's rows in increasing order
            const int row = base + u * n + 1;
            if (v[u] != v[u]) {
                nan_row = min(nan_row, row);
            } else if (v[u] > best) {
                best = v[u];
                best_row = row;
            }
        }
    }
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        nan_row = min(nan_row, __shfl_xor(nan_row, off));
        const float b2 = __shfl_xor(best, off);
        const int r2 = __shfl_xor(best_row, off);
        if (b2 > best || (b2 == best && r2 < best_row)) {
            best = b2;
            best_row = r2;
        }
    }
    const int w = tid >> 6, nw = (n + kWave - 1) / kWave;
    if ((tid & (kWave - 1)) == 0) {
        red[3 * w] = nan_row;
        red[3 * w + 1] = __builtin_bit_cast(int, best);
        red[3 * w + 2] = best_row;
    }
    __syncthreads();
    nan_row = red[0];
    best = __builtin_bit_cast(float, red[1]);
    best_row = red[2];
    for (int k = 1; k < nw; ++k) {
        nan_row = min(nan_row, red[3 * k]);
        const float b2 = __builtin_bit_cast(float, red[3 * k + 1]);
        const int r2 = red[3 * k + 2];
        if (b2 > best || (b2 == best && r2 < best_row)) {
            best = b2;
            best_row = r2;
        }
    }
    return uniform(nan_row != 0x7fffffff ? nan_row : best_row);
}

// ------------------------------------------------------------------------------------
// Generic forward of one segment by the whole workgroup: one time step per barrier, cells
// strided over the threads, rows ping-ponged in LDS.  Orders of magnitude slower than
// Forward (~1-3 ms per 30 s segment) and used only to recover a segment the fast path could
// not finish: a split segment whose cross-CU hand-off timed out (status 3 before round 2)
// and a large-vocabulary segment with more than kGatherVS distinct columns (status 2 before
// round 2).  Same arithmetic as Forward::advance (alignment.py:367-378: fp32 adds, strict
// `changed > stayed` bit, NaN-propagating max, fp64 column-0 cumsum, +inf in the last N rows
// of column 0) and the same outputs in the same places: the decision words in the launch's
// bitmap layout `lay`, the column-N history cn[0..T-1] and q0.  Returns false (nothing
// written) when two rows plus the decision words of N cells do not fit in `lds_floats`.
__device__ __noinline__ bool generic_forward(int T, int N, int blank, const float* __restrict__ E, int V,
                                             const int32_t* __restrict__ tok /* segment's tokens */,
                                             unsigned* __restrict__ bits, Layout lay, float* __restrict__ cn,
                                             float* __restrict__ q0, float* lds, int lds_floats) {
    if (3 * (N + 1) > lds_floats) return false;
    float* ra = lds;
    float* rb = lds + (N + 1);
    unsigned* wb = reinterpret_cast<unsigned*>(lds + 2 * (N + 1));  // wb[j-1]: cell j's open word
    const int tid = (int)threadIdx.x, nthr = (int)blockDim.x;
    const int inf_from = T + 1 - N;
    for (int j = tid; j <= N; j += nthr) {
        ra[j] = j == 0 ? col0_value(0, 0.0, T, N) : -INFINITY;
        if (j > 0) wb[j - 1] = 0u;
    }
    for (int t = tid; t < T; t += nthr) q0[t] = exp_cr(E[(int64_t)t * V]);
    double acc = 0.0;  // sum of em[0..t, 0] (every thread, same order)
    for (int t = 0; t < T; ++t) {
        __syncthreads();
        const float* row = E + (int64_t)t * V;
        const float eb = row[blank];
        const bool flush = (t & (kChunk - 1)) == kChunk - 1 || t == T - 1;
        const int sh = kChunk - 1 - (t & (kChunk - 1));  // keep bit 31 = first step of the block
        for (int j = tid + 1; j <= N; j += nthr) {
            int tk = tok[j - 1];
            tk = (tk >= 0 && tk < V) ? tk : 0;
            const float s = ra[j] + eb;
            const float c = ra[j - 1] + row[tk];
            unsigned w = (wb[j - 1] << 1) | (c > s ? 1u : 0u);
            rb[j] = nan_max(s, c);
            if (j == N) cn[t] = rb[j];
            if (flush) {
                int g, k;
                lay.locate(j - 1, g, k);
                bits[((int64_t)(t >> 5) * lay.C + k) * lay.lanes + g] = w << sh;
                w = 0u;
            }
            wb[j - 1] = w;
        }
        acc += (double)row[0];
        if (tid == 0) rb[0] = (t + 1 >= inf_from) ? INFINITY : (float)acc;
        float* x = ra;
        ra = rb;
        rb = x;
    }
    __syncthreads();
    return true;
}

// ------------------------------------------------------------------------------------
// Backtrack walk over the decision bitmap (alignment.py:395-421).  Uniform control flow,
// executed by the whole wave; `lay` maps cells to the bitmap's (lane, slot) words.
// Records start[k] = first frame of token k (the frame where the path moved onto it).
// Returns true on success (j reached 0), false where the reference returns None.
template <int CC, bool WT = false>  // WT: sc1 loads (kSplitWT)
__device__ __forceinline__ unsigned load_window(const unsigned* __restrict__ bits, const Layout& lay, int b, int A) {
    // Unconditional (column clamped to 1, block to 0): the walk masks invalid lanes when it
    // uses the word, so the load can stay in flight across blocks (a conditional load
    // merges into its destination and hipcc then waits for it where it is issued).
    // The block's row base is wave-uniform (scalar 64-bit math); the lane adds a 32-bit word
    // offset, so the load takes the saddr + voffset form with no per-lane 64-bit multiply.
    const unsigned* row = bits + (int64_t)uniform(max(b, 0)) * (lay.C * lay.lanes);
    const int jj = max(A - lane_id(), 1);
    int g, k;
    lay.locate<CC>(jj - 1, g, k);
    return ld_pub<WT>(row + (unsigned)(k * lay.lanes + g));
}

// Walk one 32-step block (decision indices 32b+31 .. 32b) from window offset d, run-length
// form: one iteration per token change instead of per step.  The path stays on window lane
// d until the next set bit (in walking order: increasing bit position) of that lane's word,
// moves there, and continues from the next step on lane d+1.  A successful path makes
// exactly N changes, so the serial chain costs ~N * (readlane + 8 SALU) per segment instead
// of T * 4 SALU (a per-step ballot-transposed SALU chain, replaced in round 2).  Bits of
// steps before the walk's start must be cleared.  Returns the change mask (bit 31-s = the
// path moved onto a new token at 32b+s).
__device__ __forceinline__ unsigned walk_block_rl(unsigned win, int& d) {
    // Per change: x = word[dd] & m (m: bit positions still ahead) is non-zero; p = its lowest
    // set bit is the change; m = -2 << p keeps the positions after it (0 after bit 31: the
    // walk leaves the block).  The chain is s_and -> s_ff1 -> s_lshl; the next lane's word
    // (dd does not depend on the chain) is read one change ahead so v_readlane stays off
    // it (lane dd + 1 may be past the window: read, never used).  Unrolled by four: a taken
    // branch costs more than the rest of a change (measured ~96 cycles per change for the
    // loop with one taken branch per change).
    // The lane position is not carried through the chain: every change sets one bit of cm, so
    // the walk leaves the block on lane d + popcount(cm).  Words are read two changes ahead
    // (wa / wb alternate), which keeps v_readlane's SGPR write two changes off its reader.
    unsigned cm = 0u, m = 0xFFFFFFFFu, x, wa, wb, t = (unsigned)d + 2u, p;
#define WX_RL_STEP(W, BR)                       \
    "s_ff1_i32_b32 %[p], %[x]\n\t"              \
    "s_bitset1_b32 %[cm], %[p]\n\t"             \
    "s_lshl_b32 %[m], -2, %[p]\n\t"             \
    "s_add_u32 %[t], %[t], 1\n\t"               \
    "s_and_b32 %[x], %[" #W "], %[m]\n\t"       \
    "v_readlane_b32 %[" #W "], %[win], %[t]\n\t" BR "\n\t"
    asm volatile(
        "s_add_u32 %[p], %[t], -2\n\t"
        "v_readlane_b32 %[x], %[win], %[p]\n\t"
        "s_add_u32 %[p], %[t], -1\n\t"
        "v_readlane_b32 %[wa], %[win], %[p]\n\t"
        "v_readlane_b32 %[wb], %[win], %[t]\n\t"
        "s_and_b32 %[x], %[x], %[m]\n\t"
        "s_cbranch_scc0 2f\n"
        "1:\n\t"
        WX_RL_STEP(wa, "s_cbranch_scc0 2f")
        WX_RL_STEP(wb, "s_cbranch_scc0 2f")
        WX_RL_STEP(wa, "s_cbranch_scc0 2f")
        WX_RL_STEP(wb, "s_cbranch_scc1 1b")
        "2:"
        : [t] "+s"(t), [cm] "+s"(cm), [m] "+s"(m), [x] "=&s"(x), [wa] "=&s"(wa), [wb] "=&s"(wb), [p] "=&s"(p)
        : [win] "v"(win)
        : "scc");
#undef WX_RL_STEP
    d += __popc(cm);
    return cm;
}

// The backtrack walk (alignment.py:395-421) over the decision bitmap: from (t_start, N),
// step back one frame at a time and move to the previous token where the decision bit is
// set.  Once j reaches 0 the window reads cell 0 (all zero), so blocks run to completion
// without an early-exit test.  Per block only the change mask is kept (cmask[b]);
// start frames are compacted from it afterwards.  Returns the lowest block touched, or -1
// where the reference returns None.
//
// The bitmap words are global loads (written by other waves or CUs), so the walk keeps three
// blocks' windows in flight: the window of block b - 3 is issued when block b starts, at the
// column A the walk has then; lane i loads the words of columns A - i and A - 64 - i.  The
// path moves at most 32 columns per block, so block b - 3 starts at most 64 columns left of
// A and ends within 128 of it.  At use, the 64 lanes from the walk's offset are gathered
// into one word per lane (two ds_bpermutes, skipped while the block fits the first word).
// Speculative walk segments (multi-wave workgroups, T <= kMaxLdsFrames).  The blocks below the
// top are cut into K segments of L blocks; the walker wave of segment k >= 1 starts at its top
// block from a guessed column and records its column after every block (colrec), its result
// and its end column.  Backtrack paths from different cells merge (Viterbi survivor paths),
// and the walk is a function of (block, column) alone, so once the true walk (wave 0) stands
// where segment k's walker stood after the same block — or enters segment k on its guessed
// column — the rest of that segment's change masks, end column and result are the true
// walk's, and wave 0 jumps to the segment's end.
// Decision words from the forward's bitmap (load_window): block bb's window issued at column
// A holds columns A - lane (lo) and A - 64 - lane (hi); at use the 64 lanes from the walk's
// offset are gathered (two ds_bpermutes, skipped while the block fits the first word).
template <int CC, bool WT = false>  // WT: the words were written through by other CUs (kSplitWT)
struct BitSrc {
    static constexpr bool kWT = WT;
    const unsigned* bits;
    Layout lay;
    struct Win {
        unsigned lo, hi;
        int A;
    };
    __device__ __forceinline__ void issue(Win& w, int bb, int A) const {
        w.A = uniform(A);
        w.lo = load_window<CC, WT>(bits, lay, bb, A);
        w.hi = load_window<CC, WT>(bits, lay, bb, A - 64);
    }
    __device__ __forceinline__ void end_block(int) const {}
    __device__ __forceinline__ void window(const Win& w, int b, int j, unsigned& win, int& dd) const {
        (void)b;
        const int lane = lane_id();
        const int d = uniform(w.A - j);  // 0 .. 96
        if (d <= 31) {
            win = (w.A - lane >= 1) ? w.lo : 0u;
            dd = d;
        } else {
            const int o = d + lane;  // column w.A - o
            const unsigned a = (unsigned)__shfl((int)w.lo, o & 63);
            const unsigned h = (unsigned)__shfl((int)w.hi, o & 63);
            win = (w.A - o >= 1 && o < 128) ? (o < 64 ? a : h) : 0u;
            dd = 0;
        }
    }
};

// Decision words recomputed from checkpoint rows (MODE 2 kernels).  The backtrack test at
// (t, j) is the forward's comparison `tr[t-1, j-1] + em[t-1, tok[j-1]] > tr[t-1, j] + em[t-1,
// blank]` (alignment.py:372-378, :400-404), and fp32 adds and maxima are deterministic, so the
// forward's decisions are recomputed bit for bit from the row it started the chunk with.  A
// block's path enters at column j and leaves at >= j - 32, so its words are needed for columns
// j - 32 .. j; over 32 steps a cell depends on the 32 cells to its left, so the band is the
// 64 lanes L -> column j - 63 + L started from checkpoint row 32b plus column j - 64 as lane 0's
// first left input: lane L's decision at step k is exact when L >= k (lane 0's later left
// inputs are unknown), i.e. columns >= j - 32 at every step.  Column 0 (tr[t][0], :367-370)
// is not a cell: where the band reaches it, its lane is set every step from the fp64 cumsum
// (checkpointed per chunk) in the reference's order.
//
// The block's 32 emission rows are staged per wave into an LDS slot ([32][VS], row stride VS
// so the per-step reads take immediate offsets) by LDS-DMA.  A walker with two slots (one-wave
// kernels: the forward's two buffers) loads the next block's rows into the other slot while it
// computes; one slot per walker (multi-wave kernels) loads its rows at use and warms the L2
// with the next block's rows (a DMA into a shared scratch row nobody reads).  The checkpoint
// values and token ids of the window are loaded with the walk's three-block prefetch (columns
// A - lane, A - 64 - lane, A - 128 - lane: the band of a block entered within 96 columns of A).
template <int CC, int VS>
struct CkSrc {
    static constexpr bool kWT = false;
    const float* ck;      // checkpoint rows: tr[32q][j] at cell j's bitmap word of block q
    Layout lay;
    const double* acc;    // [q]: sum of em[0 .. 32q - 1, 0] in fp64 (column 0 before row 32q)
    const float* E;       // segment's emission rows [T, V]
    const int32_t* tok;   // segment's tokens
    int T, N, V, blank;
    bool x4;              // V == 32 and 16-byte aligned rows: 8 rows per DMA instruction
    float* slot[2];       // LDS [kChunk][VS] slots of this wave (slot[1] == slot[0]: one slot)
    float* junk;          // LDS: 1 KB the L2 warm-up DMA writes
    int cur = 0, rdy_blk = -1000;  // slot holding block rdy_blk's rows, landed
    struct Win {
        float c0, c1, c2;  // checkpoint row of block bb: columns A - lane, A - 64 - lane, A - 128 - lane
        int k0, k1, k2;    // token ids of the same columns
        int A;
    };
    __device__ __forceinline__ float ck_of(const float* row, int col) const {
        col = max(col, 1);  // (columns <= 0: a don't-care lane)
        int g, k;
        lay.locate<CC>(col - 1, g, k);
        return row[(unsigned)(k * lay.lanes + g)];
    }
    __device__ __forceinline__ int tok_of(int col) const { return tok[max(col, 1) - 1]; }
    __device__ __forceinline__ void issue(Win& w, int bb, int A) const {
        w.A = uniform(A);
        const int lane = lane_id();
        const int bc = uniform(max(bb, 0));
        const float* row = ck + (int64_t)bc * (lay.C * lay.lanes);
        w.c0 = ck_of(row, A - lane);
        w.c1 = ck_of(row, A - 64 - lane);
        w.c2 = ck_of(row, A - 128 - lane);
        w.k0 = tok_of(A - lane);
        w.k1 = tok_of(A - 64 - lane);
        w.k2 = tok_of(A - 128 - lane);
    }
    // LDS-DMA of block b's rows (clamped into the segment) to dst, or all onto the junk row
    __device__ __forceinline__ void dma_rows(int b, float* dst, bool warm) const {
        const int l = lane_id();
        const int r0 = max(b, 0) * kChunk;
        const unsigned base = (unsigned)uniform((int)lds_addr(warm ? junk : dst));
        if (VS == 32 && x4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = min(r0 + 8 * i + (l >> 3), T - 1);
                glds_dwordx4(E, (unsigned)(r * 32 + (l & 7) * 4) * 4u, base + (warm ? 0u : (unsigned)(i * 1024)));
            }
        } else if (l < V) {
            for (int r = 0; r < kChunk; ++r) {
                const int t = min(r0 + r, T - 1);
                glds_dword(E + (int64_t)t * V, (unsigned)l * 4u, base + (warm ? 0u : (unsigned)(r * VS * 4)));
            }
        }
    }
    // The slot holding block b's rows.  Two slots: block b - 1's rows go into the other slot now
    // and are waited for at the end of block b (end_block), a block later.  One slot: the L2 is
    // warmed with block b - 1's rows now; end_block loads them into the slot once block b's
    // recompute has read it.  (Waiting for a DMA here would also wait for the window loads the
    // walk issued at the end of the previous block: an HBM round trip per block.)
    __device__ __forceinline__ const float* stage(int b) {
        const bool two = slot[1] != slot[0];
        if (uniform(rdy_blk) != b) {  // (the first block, or after a jump)
            cur = 0;
            dma_rows(b, slot[0], false);
            wait_vm();
            rdy_blk = b;
        }
        const float* s = cur ? slot[1] : slot[0];  // (no dynamic index: it would put the struct in scratch)
        if (two)
            dma_rows(b - 1, cur ? slot[0] : slot[1], false);
        else
            dma_rows(b - 1, nullptr, true);
        return s;
    }
    // block b walked: the next block's rows ready before the walk issues its next window loads
    __device__ __forceinline__ void end_block(int b) {
        if (slot[1] != slot[0]) {
            wait_vm();
            cur ^= 1;
        } else {
            dma_rows(b - 1, slot[0], false);
            wait_vm();
        }
        rdy_blk = b - 1;
    }
    __device__ __forceinline__ void window(const Win& w, int b, int j, unsigned& win, int& dd) {
        const int lane = lane_id();
        const int d = uniform(w.A - j);  // 0 .. 96
        const float* slotp = stage(b);
        // band lane L: column j - 63 + L, at window offset o = d + 63 - L
        const int o = d + 63 - lane;
        const float x0 = __shfl(w.c0, o & 63), x1 = __shfl(w.c1, o & 63), x2 = __shfl(w.c2, o & 63);
        const int y0 = __shfl(w.k0, o & 63), y1 = __shfl(w.k1, o & 63), y2 = __shfl(w.k2, o & 63);
        float v = o < 64 ? x0 : (o < 128 ? x1 : x2);
        int tk = o < 64 ? y0 : (o < 128 ? y1 : y2);
        tk = (tk >= 0 && tk < V) ? tk : 0;
        const int o0 = d + 64;  // column j - 64: lane 0's first left input
        // (column 0 when j == 64: not a checkpointed cell)
        const float left0 = j == 64 ? col0_value(b * kChunk, acc[max(b, 0)], T, N)
                                    : uniformf(o0 < 128 ? __shfl(w.c1, o0 & 63) : __shfl(w.c2, o0 & 63));
        const char* sb = reinterpret_cast<const char*>(slotp);
        const int toff = tk * 4, boff = blank * 4;
        unsigned bits = 0u;
        // 32 steps in groups of four, the next group's LDS operands read ahead (sched_barrier
        // keeps hipcc from hoisting all the reads: registers are the forward's occupancy).
        // HAS_C0: column 0 is band lane 63 - j (j <= 63), set every step from the cumsum.
        auto steps = [&](auto has_c0_tag) {
            constexpr bool HAS_C0 = decltype(has_c0_tag)::value;
            const bool c0 = HAS_C0 && lane == 63 - j;
            double a = HAS_C0 ? acc[max(b, 0)] : 0.0;  // (rare: a load in the chain is fine)
            const int t0 = b * kChunk;
            if (c0) v = col0_value(t0, a, T, N);
            float eb[4], et[4], e0[4];
            auto rd = [&](int k0, float(&xb)[4], float(&xt)[4], float(&x0)[4]) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    xb[u] = *reinterpret_cast<const float*>(sb + boff + (k0 + u) * VS * 4);
                    xt[u] = *reinterpret_cast<const float*>(sb + toff + (k0 + u) * VS * 4);
                    if (HAS_C0) x0[u] = *reinterpret_cast<const float*>(sb + (k0 + u) * VS * 4);
                }
            };
            rd(0, eb, et, e0);
#pragma unroll
            for (int g = 0; g < kChunk / 4; ++g) {
                float nb[4], nt[4], n0[4];
                if (g + 1 < kChunk / 4) rd(4 * (g + 1), nb, nt, n0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = 4 * g + u;
                    const float left = k == 0 ? dpp_shr1(left0, v)
                                              : __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                                              __builtin_bit_cast(int, v), 0x138 /* wave_shr:1 */,
                                                                              0xF, 0xF, true));
                    const float st = v + eb[u];
                    const float ch = left + et[u];
                    bits = shift_in(bits, ch, st);
                    v = nan_max(st, ch);
                    if constexpr (HAS_C0) {
                        a += (double)e0[u];
                        if (c0) v = col0_value(t0 + k + 1, a, T, N);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    eb[u] = nb[u];
                    et[u] = nt[u];
                    if (HAS_C0) e0[u] = n0[u];
                }
            }
        };
        if (j > 63)
            steps(BoolTag<false>{});
        else
            steps(BoolTag<true>{});
        // lane i of the walk's window = column j - i = band lane 63 - i
        const unsigned r = (unsigned)__shfl((int)bits, 63 - lane);
        win = (j - lane >= 1) ? r : 0u;
        dd = 0;
    }
};

struct SpecWalk {
    int K, L0, Lb, ex, top;  // segments; blocks of segment 0 (L0), of the others (Lb, +1 for k <= ex)
    const int* colrec;  // LDS, per block: the segment walker's column after it (-1: not reached)
    const int* gstart;  // LDS [K]: guessed column at the top of segment k
    const int* sres;    // LDS [K]: the walker's result (-2: the path continues below the segment)
    const int* send;    // LDS [K]: its column after the segment's last block
    // after the barrier: gstart / sres / send of segment `lane` in lane `lane` (read by
    // v_readlane: the merge chain was a serial LDS round trip per segment)
    int vg, vr, ve;
    __device__ __forceinline__ int gst(int k) const { return __builtin_amdgcn_readlane(vg, k); }
    __device__ __forceinline__ int res(int k) const { return __builtin_amdgcn_readlane(vr, k); }
    __device__ __forceinline__ int end(int k) const { return __builtin_amdgcn_readlane(ve, k); }
    // segment k covers blocks lo(k) .. lo(k - 1) - 1 (segment 0: up to top); lo(K - 1) = 0
    __device__ __forceinline__ int lo(int k) const {
        return k == 0 ? top - L0 + 1 : max(top - L0 - (k * Lb + min(k, ex)) + 1, 0);
    }
};

// The backtrack walk (alignment.py:395-421) over the decision bitmap: from column j at the
// top of block b (steps above the start cleared by first_mask), step back one frame at a time
// and move to the previous token where the decision bit is set.  Once j reaches 0 the window
// reads cell 0 (all zero), so blocks run to completion without an early-exit test.  Per
// block only the change mask is kept (cmask[b]); start frames are compacted from it
// afterwards.  Returns the block where j reached 0, -1 where the reference returns None
// (block 0 done with j > 0), or -2 when it stopped after block b_stop > 0 with the path
// going on (column in j_out).  colrec (LDS, optional) receives the column after each block;
// spec (optional) lets the walk jump over blocks a merged segment walker has done.
//
// The bitmap words are global loads (written by other waves or CUs), so the walk keeps three
// blocks' windows in flight: the window of block b - 3 is issued when block b starts, at the
// column A the walk has then; lane i loads the words of columns A - i and A - 64 - i.  The
// path moves at most 32 columns per block, so block b - 3 starts at most 64 columns left of
// A and ends within 128 of it.  At use, the 64 lanes from the walk's offset are gathered
// into one word per lane (two ds_bpermutes, skipped while the block fits the first word).
//
// Src is where the decision words come from: BitSrc reads the forward's bitmap, CkSrc (the
// checkpointed throughput kernels) recomputes each block's band from the forward's checkpoint
// rows.  Src::issue(w, bb, A) starts block bb's loads for a walk standing at column A;
// Src::window(w, b, j, win, dd) makes win = the block's words with lane dd + i = column j - i.
template <class Src>
__device__ __forceinline__ int walk_range(Src& src, int j, int b, unsigned first_mask, int b_stop,
                                          unsigned* cmask, bool cmask_in_lds, int* colrec, const SpecWalk* spec,
                                          int& j_out, int wtop = 0x7fffffff, int* jentry = nullptr) {
    using Win = typename Src::Win;
    typedef __attribute__((address_space(3))) int lds_int;
    const int lane = lane_id();
    b = uniform(b);
    j = uniform(j);
#ifdef WX_PHASE_TIMING
    unsigned long long t_rl = 0, n_ch = 0, n_bl = 0, t_win = 0;
    auto dump = [&]() {
        if (threadIdx.x == 0 && blockIdx.x < 8192) {  // (wave 0's last walk_range)
            unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + 13) * 3;
            o[0] = t_rl;
            o[1] = n_ch;
            o[2] = n_bl;
        }
        const int wv_ = (int)threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0 && wv_ < 8 && blockIdx.x < 8192) {  // slots 16 + wave (24: wave 0's second walk)
            unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + (spec ? 24 : 16 + wv_)) * 3;
            o[0] = t_win;  // cycles in the window gather (its load wait)
            o[1] = t_rl;   // in the run-length loop
            o[2] = n_bl;   // blocks
        }
    };
#else
    auto dump = [] {};
#endif
    unsigned cmv = 0u;    // change masks of blocks gb + lane
    int gtop = b & 63;    // highest lane of the current group the walk has written
    int sk = 0, slo = spec ? spec->lo(0) : 0;  // segment of the current block, its lowest block
    auto flush = [&](int bb) {  // store the group's masks written since the last flush (blocks >= bb)
        const int gb = bb & ~63;
        if (lane >= (bb & 63) && lane <= gtop && gb + lane <= wtop) {
            if (cmask_in_lds)
                ((__attribute__((address_space(3))) unsigned*)cmask)[gb + lane] = cmv;
            else
                ((__attribute__((address_space(1))) unsigned*)cmask)[gb + lane] = cmv;
        }
        gtop = 63;
    };
    auto issue = [&](Win& w, int bb, int A) { src.issue(w, bb, A); };
    // walks block b with window w (wn, wa: the next two blocks' windows, re-issued after a
    // jump); false when the walk is over (result in res)
    auto block = [&](Win& w, Win& wn, Win& wa, int& res) -> bool {
        unsigned win;
        int dd;
#ifdef WX_PHASE_TIMING
        WX_T(wi0);
#endif
        src.window(w, b, j, win, dd);
        win &= first_mask;
#ifdef WX_PHASE_TIMING
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        WX_T(wi1);
        t_win += wi1 - wi0;
#endif
        first_mask = 0xFFFFFFFFu;
        const int d0 = dd;
#ifdef WX_PHASE_TIMING
        WX_T(rl0);
#endif
        const unsigned cm = walk_block_rl(win, dd);
#ifdef WX_PHASE_TIMING
        WX_T(rl1);
        t_rl += rl1 - rl0;
        n_ch += __popc(cm);
        ++n_bl;
#endif
        // change masks are collected in lane b % 64 and stored 64 blocks at a time, through
        // an explicit LDS or global store (a flat store in the loop makes hipcc drain every
        // pending load at each wait)
        cmv = lane == (b & 63) ? cm : cmv;
        j = uniform(j - (dd - d0));
        if (b > wtop) {  // (blocks above wtop: walked, not recorded)
            if (b == wtop + 1) *jentry = j;
        } else if (colrec && lane == 0) {
            ((lds_int*)colrec)[b] = j;
        }
        bool done = j <= 0 || b == 0 || b == b_stop;
        int r = j <= 0 ? b : (b == 0 ? -1 : -2);
        if (spec && !done) {
            // merged with a segment walker: mid-segment on its recorded column, or at a segment's
            // top on its guessed column; follow merged segments to the first one that is not
            while (b < slo) slo = spec->lo(++sk);  // (b only moves down)
            int k = sk;
            int bb = b, jj = j;
            bool merged = k >= 1 && bb != spec->lo(k) && jj == uniform(((const lds_int*)spec->colrec)[bb]);
            for (;;) {
                if (merged) {
                    r = spec->res(k);
                    bb = spec->lo(k);
                    jj = spec->end(k);
                    if (r != -2) break;
                }
                merged = bb == spec->lo(k) && k + 1 < spec->K && jj == spec->gst(k + 1);
                if (!merged) break;
                ++k;
            }
            if (bb != b) {  // jumped: the walk goes on after block bb (or is over: r)
                flush(b);
                if (r != -2) {
                    res = r;
                    dump();
                    return false;
                }
                b = uniform(bb);
                j = uniform(jj);
                gtop = (b - 1) & 63;
                issue(w, b - 3, j);
                issue(wn, b - 1, j);
                issue(wa, b - 2, j);
                --b;
                return true;
            }
        }
        if (done || (b & 63) == 0) flush(b);
        src.end_block(b);
        issue(w, b - 3, j);  // unconditional (a conditional refill would merge and wait)
        if (done) {
            res = r;
            j_out = j;
            dump();
            return false;
        }
        --b;
        return true;
    };
    Win w0, w1, w2;
    issue(w0, b, j);
    issue(w1, b - 1, j);
    issue(w2, b - 2, j);
    int res = -1;
    for (;;) {
        if (!block(w0, w1, w2, res)) return res;
        if (!block(w1, w2, w0, res)) return res;
        if (!block(w2, w0, w1, res)) return res;
    }
}

template <class Src>
__device__ __forceinline__ int walk_impl(Src& src, int N, int t_start, unsigned* cmask, bool cmask_in_lds) {
    if (t_start <= 0 || N <= 0) return -1;
    int jo;
    return walk_range(src, N, (t_start - 1) >> 5, 0xFFFFFFFFu << (31 - ((t_start - 1) & 31)), 0, cmask,
                      cmask_in_lds, nullptr, nullptr, jo);
}

template <int CC>  // cells per lane of the bitmap layout (0: runtime lay.C)
__device__ int walk(const unsigned* __restrict__ bits, const Layout& lay, int N, int t_start, unsigned* cmask,
                    bool cmask_in_lds) {
    BitSrc<CC> src{bits, lay};
    return walk_impl(src, N, t_start, cmask, cmask_in_lds);
}

// Speculative walk: blocks top..0 of a walk from (t_start, N) in K segments over the workgroup's
// first K waves (SpecWalk).  Phase 1: wave 0 walks the top segment; wave k starts kSpecOverlap
// blocks above its segment from a guessed column and walks those blocks unrecorded, so that
// its path has usually merged with the true one when it enters the segment (its entry column
// is gstart[k]).  Phase 2 (after a workgroup barrier): wave 0 goes on from the top segment's
// end, jumping over whatever merged — usually every segment, with no block walked again.
// Every wave of the workgroup calls it (the barrier); returns wave 0's result (the lowest
// block, or -1), meaningful in wave 0.
constexpr int kSpecMinBlocks = 4;  // blocks per segment at least
constexpr int kSpecOverlap = 2;  // unrecorded blocks a walker starts above its segment (A/B: 1, 3, 4 slower)
// wave 0's t_start search, in walk blocks (A/B: 1, 3 or 5 within noise)
constexpr int kSpecArgmaxBlocks = 3;
template <class Src>
__device__ __forceinline__ int walk_spec(Src& lw, int N, int T, const float* cn, unsigned* cmask, bool cmask_in_lds,
                                         int K, int* colrec, int* sbuf, int& t_start) {
    // (one walk_range call site before the barrier and one after: every call site inlines a
    // copy of the walk, and the checkpointed walk's blocks are long)
    const int wv = uniform((int)threadIdx.x >> 6);
    const int lane = lane_id();
    SpecWalk sw;
    sw.K = K;
    sw.colrec = colrec;
    sw.gstart = sbuf;
    sw.sres = sbuf + K;
    sw.send = sbuf + 2 * K;
    int res = -1, jo = 0, tb = 0;
    unsigned fm = 0u;
    // The segments cover the blocks below T (t_start <= T): the walkers start while wave 0
    // alone finds t_start, so its segment is kSpecArgmaxBlocks shorter than theirs.  (Round 2
    // waited for a workgroup-wide t_start first: 1-2 us slower.)  K == 1: wave 0 walks alone.
    // Balanced: wave 0 takes its share less the argmax allowance, the other K - 1 segments
    // split the rest within one block of each other (a uniform length had left the last
    // walker a single block while the others walked 7 + kSpecOverlap).
    sw.top = (T - 1) >> 5;
    const int nb = sw.top + 1;
    sw.L0 = max((nb + kSpecArgmaxBlocks + K / 2) / K - kSpecArgmaxBlocks, 1);
    if (K > 1 && nb - sw.L0 < K - 1) K = max(nb - sw.L0 + 1, 1);  // (one block per walker at least)
    if (K <= 1 || sw.L0 >= nb) {
        K = 1;
        sw.L0 = nb;
        sw.Lb = 1;
        sw.ex = 0;
    } else {
        sw.Lb = (nb - sw.L0) / (K - 1);
        sw.ex = (nb - sw.L0) % (K - 1);
    }
    sw.K = K;
    sw.sres = sbuf + K;
    sw.send = sbuf + 2 * K;
    const int tref = T;
#ifdef WX_PHASE_TIMING
    WX_T(sp0);
    unsigned long long sp_am = sp0;
#endif
    // this wave's first walk: wave 0 the top segment from (t_start, N); wave k < K its segment
    // from a guessed column kSpecOverlap blocks above it
    bool go = false;
    int j0 = N, b0 = 0, stop = 0, top = 0x7fffffff, je = -1;
    unsigned fm0 = 0xFFFFFFFFu;
    int* rec = nullptr;
    if (wv == 0) {
        t_start = column_argmax<Src::kWT>(cn, T);
#ifdef WX_PHASE_TIMING
        sp_am = __builtin_amdgcn_s_memtime();
#endif
        if (t_start <= 0) {
            res = -1;  // (the reference's None)
        } else {
            tb = (t_start - 1) >> 5;
            fm = 0xFFFFFFFFu << (31 - ((t_start - 1) & 31));
            go = tb >= sw.lo(0);
            res = -3;  // (starts in a lower segment: after the barrier)
            b0 = tb;
            fm0 = fm;
            stop = sw.lo(0);
        }
    } else if (wv < K) {
        top = sw.lo(wv - 1) - 1;
        const int lo = sw.lo(wv), sb = top + kSpecOverlap;
        // guess: the straight line from (0, 0) to (tref, N), inside the cells the path can
        // occupy at time 32 (sb + 1) (column <= time, N - column <= remaining steps)
        const int tt = 32 * (sb + 1);
        int g = (int)(((int64_t)N * tt + tref / 2) / tref);
        g = min(max(g, max(1, N - (tref - tt))), min(N, tt));
        for (int bb = lo + lane; bb <= top; bb += kWave) colrec[bb] = -1;
        go = true;
        j0 = g;
        b0 = sb;
        stop = lo;
        rec = colrec;
    }
    if (go) {
        const int r = walk_range(lw, j0, b0, fm0, stop, cmask, cmask_in_lds, rec, nullptr, jo, top, &je);
        if (wv == 0) {
            res = r;
        } else if (lane == 0) {  // je: column entering the segment (-1: the path ended above it)
            sbuf[wv] = je;
            sbuf[K + wv] = r;
            sbuf[2 * K + wv] = jo;
        }
    }
#ifdef WX_PHASE_TIMING
    WX_T(sp1);
#endif
    wave_fence();
    block_fence();
#ifdef WX_PHASE_TIMING
    WX_T(sp2);
    // per wave (slots 6 + wave): wave 0 [argmax, first walk, barrier] cycles since entry; walkers
    // [first walk, barrier, K]
    if (lane == 0 && wv <= 6 && blockIdx.x < 8192) {
        unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + 6 + wv) * 3;
        o[0] = wv == 0 ? sp_am - sp0 : sp1 - sp0;
        o[1] = wv == 0 ? sp1 - sp0 : sp2 - sp0;
        o[2] = wv == 0 ? sp2 - sp0 : (unsigned long long)K;
    }
#endif
    if (wv == 0 && (res == -2 || res == -3)) {
        int j1 = N, b1 = tb;
        unsigned fm1 = fm;
        const int kl = min(lane, K - 1);  // (K <= waves <= 64)
        sw.vg = sbuf[kl];
        sw.vr = sbuf[K + kl];
        sw.ve = sbuf[2 * K + kl];
        if (res == -2) {
            // segments entered on their guessed column are the true walk's as a whole
            int k = 1;
            for (; k < K && jo == sw.gst(k); ++k) {
                res = sw.res(k);
                jo = sw.end(k);
                if (res != -2) return res;
            }
            j1 = jo;
            b1 = sw.lo(k - 1) - 1;
            fm1 = 0xFFFFFFFFu;
        }
        res = walk_range(lw, j1, b1, fm1, 0, cmask, cmask_in_lds, nullptr, &sw, jo);
    }
    return res;
}

// start[k] = k-th change frame in increasing time: a popcount prefix over the change masks
// of blocks [b_lo, b_hi] (wave 0).
__device__ void compact_starts(const unsigned* cmask, int b_lo, int b_hi, int32_t* __restrict__ start) {
    const int lane = lane_id();
    int base = 0;
    for (int b0 = b_lo; b0 <= b_hi; b0 += kWave) {
        const int b = b0 + lane;
        const unsigned m = (b <= b_hi) ? cmask[b] : 0u;
        const int c = __popc(m);
        int incl = c;  // inclusive wave scan of popcounts
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        int k = base + incl - c;
        unsigned mm = m;
        while (mm) {  // bit 31 = lowest frame of the block
            const int p = 31 - __clz(mm);
            start[k++] = b * kChunk + (31 - p);
            mm &= ~(1u << p);
        }
        base += __shfl(incl, kWave - 1);
    }
}

// compact_starts with every wave of the workgroup (every thread calls it): lane b of each
// 64-block group holds block b's mask and its exclusive popcount prefix; wave w stores the
// bits at positions 31 - w, 31 - w - nw, ... (token k = prefix + the set bits above the
// position: frames earlier in the block), so each wave makes 32 / nw conditional stores
// instead of wave 0 looping over every set bit of a block (1.2 us of config 2's tail).
__device__ void compact_starts_par(const unsigned* cmask, int b_lo, int b_hi, int32_t* __restrict__ start) {
    const int lane = lane_id();
    const int wv = uniform((int)threadIdx.x >> 6), nw = (int)blockDim.x >> 6;
    int base = 0;
    for (int b0 = b_lo; b0 <= b_hi; b0 += kWave) {
        const int b = b0 + lane;
        const unsigned m = (b <= b_hi) ? cmask[b] : 0u;
        const int c = __popc(m);
        int incl = c;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        const int k0 = base + incl - c;
        for (int p = 31 - wv; p >= 0; p -= nw) {  // bit 31 = lowest frame of the block
            const unsigned hi = p == 31 ? 0u : m >> (p + 1);
            if ((m >> p) & 1u) start[k0 + __popc(hi)] = b * kChunk + (31 - p);
        }
        base += __shfl(incl, kWave - 1);
    }
}

// merge_repeats from per-token start frames (alignment.py:438-454 + the prob rule of :409).
__device__ void merge_tokens(const float* __restrict__ E, int V, const int32_t* __restrict__ tok, int N, int t_start,
                             const float* __restrict__ q0, const int32_t* __restrict__ start, int32_t* __restrict__ seg_end,
                             double* __restrict__ seg_score) {
    for (int k = (int)threadIdx.x; k < N; k += (int)blockDim.x) {
        const int s = start[k];
        const int e = (k + 1 < N) ? start[k + 1] : t_start;
        int tk = tok[k];
        tk = (tk >= 0 && tk < V) ? tk : 0;
        double sum = (double)exp_cr(E[(int64_t)s * V + tk]);
        int x = s + 1;
        for (; x + 8 <= e; x += 8) {  // 8 loads in flight, adds in the reference's order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = q0[x + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) sum += (double)v[u];
        }
        for (; x < e; ++x) sum += (double)q0[x];
        seg_end[k] = e;
        seg_score[k] = sum / (double)(e - s);
    }
}

// merge_tokens with the segment's q0 row and start frames staged in LDS first (coalesced, 8
// loads in flight per thread), so each token's left-to-right fp64 sum reads LDS instead of
// a chain of dependent global loads; each token's first-frame emission is loaded one token
// ahead.  Needs T + N floats of `lds`; every thread of the workgroup calls it.
__device__ void merge_tokens_lds(const float* __restrict__ E, int V, const int32_t* __restrict__ tok, int N, int T,
                                 int t_start, const float* __restrict__ q0, const int32_t* __restrict__ start,
                                 int32_t* __restrict__ seg_end, double* __restrict__ seg_score, float* lds) {
    float* qs = lds;
    int* ss = reinterpret_cast<int*>(lds + T);
    const int tid = (int)threadIdx.x, nthr = (int)blockDim.x;
    constexpr int kB = 8;
    for (int base = tid; base < T; base += kB * nthr) {
        float v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) v[u] = q0[min(base + u * nthr, T - 1)];
#pragma unroll
        for (int u = 0; u < kB; ++u)
            if (base + u * nthr < T) qs[base + u * nthr] = v[u];
    }
    for (int base = tid; base < N; base += kB * nthr) {
        int v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) v[u] = start[min(base + u * nthr, N - 1)];
#pragma unroll
        for (int u = 0; u < kB; ++u)
            if (base + u * nthr < N) ss[base + u * nthr] = v[u];
    }
    block_fence();
    auto first = [&](int k) {  // em[start_k, tok_k] (clamped: an unconditional load)
        const int kk = min(k, N - 1);
        int tk = tok[kk];
        tk = (tk >= 0 && tk < V) ? tk : 0;
        return E[(int64_t)ss[kk] * V + tk];
    };
    float e_next = first(tid);
    for (int k = tid; k < N; k += nthr) {
        const float e_cur = e_next;
        e_next = first(k + nthr);
        const int s = ss[k];
        const int e = (k + 1 < N) ? ss[k + 1] : t_start;
        double sum = (double)exp_cr(e_cur);
        for (int x = s + 1; x < e; ++x) sum += (double)qs[x];
        seg_end[k] = e;
        seg_score[k] = sum / (double)(e - s);
    }
}

// Order one wave's own global/LDS writes before its later reads by other lanes (no
// barrier: safe inside wave-divergent regions of multi-wave workgroups).

// (cells per lane C, DP waves per segment W, helper wave H) buckets, one kernel
// instantiation each; id = C << 8 | W << 1 | H.
// Throughput mode (many segments in flight): one wave per segment up to N = 512; longer
// transcripts use W waves of 8 cells per lane with a chunk halo (Geometry): at most ~124
// VGPRs keeps 4 waves per SIMD, which beat one wide (16-32 cells per lane) wave per
// segment by 4-10% on T = 3000, N = 900 batches.  Latency mode (few segments: the
// chip would otherwise be mostly idle): a segment's columns are spread over 3 or 7 waves
// plus the helper (at most 2 waves per SIMD, which still issue at the full rate), so each
// wave issues fewer instructions per time step.  (Waves beyond column N only keep the
// barrier count, so a wide bucket costs no time: 30 s segments, N 257..704, share one.)
#define WX_BUCKETS(X)                                                                                    \
    X(1, 1, 0) X(2, 1, 0) X(4, 1, 0) X(6, 1, 0) X(8, 1, 0) X(8, 2, 0) X(8, 4, 0) X(8, 8, 0) X(16, 8, 0) \
        X(32, 8, 0) X(1, 3, 1) X(1, 7, 1) X(2, 7, 1) X(4, 7, 1) X(8, 7, 1)

__host__ __device__ constexpr int bucket_make(int C, int W, int H) { return (C << 8) | (W << 1) | H; }
__host__ __device__ constexpr int bucket_C(int id) { return id >> 8; }
__host__ __device__ constexpr int bucket_W(int id) { return (id >> 1) & 127; }

__host__ __device__ constexpr int bucket_capacity(int C, int W) {
    return C * (kWave + (W - 1) * (kWave - (W > 1 ? (32 + C - 1) / C : 0)));
}

// Buckets of each mode in increasing capacity (compare chains: a dynamically indexed
// table would live in scratch on the device).
#define WX_PICK(CC, WW, HH) \
    if (N <= bucket_capacity(CC, WW)) return bucket_make(CC, WW, HH);
__host__ __device__ __forceinline__ int bucket_id(int N, int mode = 0) {
    if (mode == 1) {
        WX_PICK(1, 1, 0) WX_PICK(1, 3, 1) WX_PICK(1, 7, 1) WX_PICK(2, 7, 1) WX_PICK(4, 7, 1) WX_PICK(8, 7, 1)
        WX_PICK(16, 8, 0)
    } else {
        WX_PICK(1, 1, 0) WX_PICK(2, 1, 0) WX_PICK(4, 1, 0) WX_PICK(6, 1, 0) WX_PICK(8, 1, 0) WX_PICK(8, 2, 0)
        WX_PICK(8, 4, 0) WX_PICK(8, 8, 0) WX_PICK(16, 8, 0)
    }
    return bucket_make(32, 8, 0);
}
#undef WX_PICK

// bitmap words per 32-step block of a segment in bucket `id`
__host__ __device__ __forceinline__ int bucket_cells_total(int id) { return bucket_C(id) * kWave * bucket_W(id); }

// Split buckets (C cells per lane, W DP waves + 1 helper per part, P parts): the chunk
// halo runs through all W * P virtual waves.  Segments too long for the widest split bucket
// use the single-CU latency buckets in the same launch.
// (A/B, config 2: 5 DP waves per part instead of 4 were 2 us slower, 6 — two hand-off hops
// fewer — 0.8 us faster, though the DP waves sharing a SIMD slow each other's chains.)
#define WX_SPLIT_BUCKETS(X) X(1, 3) X(1, 4) X(2, 3) X(4, 3)
constexpr int kSplitFlag = 1 << 20;
__host__ __device__ constexpr int split_capacity(int C, int W, int P) {
    return C * (kWave + (W * P - 1) * (kWave - (32 + C - 1) / C));
}
#define WX_PICK_SPLIT(CC, WW) \
    if (N <= split_capacity(CC, WW, P)) return bucket_make(CC, WW, 1) | kSplitFlag;
__host__ __device__ __forceinline__ int split_bucket_id(int N, int P) {
    WX_SPLIT_BUCKETS(WX_PICK_SPLIT)
    return bucket_id(N, 1);
}
#undef WX_PICK_SPLIT

// A split launch runs ONE split kernel (the bucket of the batch's longest segment): its
// grid is S * P workgroups, one per CU, and a second split grid would queue behind it
// (measured: workgroups of the second kernel started up to 70 us late).  Shorter segments
// leave that bucket's extra waves idle.  Segments beyond its capacity use the single-CU
// latency buckets.
__host__ __device__ __forceinline__ int split_capacity_of(int id, int P) {
    return split_capacity(bucket_C(id & ~kSplitFlag), bucket_W(id & ~kSplitFlag), P);
}
// Layout::make needs N >= ceil(N/C) * (C-1) (at most one missing cell per lane); the
// per-N buckets always satisfy it, a launch-wide split bucket may not for short segments,
// which then take a throughput bucket (one wave, small LDS: it shares CUs with the parts).
__host__ __device__ constexpr bool layout_fits(int N, int C) { return N >= (N + C - 1) / C * (C - 1); }
__host__ __device__ __forceinline__ int launch_split_bucket(int N, int P, int split_id) {
    if (N > split_capacity_of(split_id, P)) return bucket_id(N, 1);
    return layout_fits(N, bucket_C(split_id & ~kSplitFlag)) ? split_id : bucket_id(N, 0);
}

struct AlignArgs {
    const float* em;
    const int64_t* em_off;
    int V;
    const int32_t* tok;
    const int64_t* tok_off;
    const int32_t* blank_id;
    int S;
    int mode;  // 0 throughput buckets, 1 latency buckets
    int x4;    // V == 32 and 16-byte aligned rows: 16-byte LDS staging
    int32_t* seg_start;
    int32_t* seg_end;
    double* seg_score;
    int32_t* t_start;
    int32_t* status;
    unsigned* bits;  // workspace: bitmap region
    int bits_stride_cells;  // 64 * Cstride dwords per block
    float* q0;       // workspace: sum_T floats
    unsigned* cmask; // workspace: walk change masks, (floor(row0/32) + seg) words per segment
    double* c0acc;   // workspace (MODE 2): column-0 fp64 cumsum per chunk, same offsets as cmask
    float* cn;       // workspace: column N history, segment at (row0 + 4 seg) & ~3
    int parts;       // split launches: workgroups (CUs) per segment, else 1
    int split_id;    // split launches: the one split bucket (segments up to its capacity)
    unsigned epoch;  // split launches: per-launch tag of the hand-off granules and counters
    uint64_t* xg;    // workspace: hand-off granules, (floor(row0/32) + seg + q) * 3 * 40
    uint64_t* arrive;// workspace: per-segment arrival counters {count, epoch} (split_arrive)
    int spin;        // split launches: hand-off re-reads before a part counts as lost
    int flags;       // split launches: kArgFenced | kArgXcdSpread (WX_SPLIT_FENCED, WX_SPLIT_XCD_SPREAD)
};

// Per-segment arrival of a split segment's parts.  The counter is one 8-byte word,
// {low: count | 0x80 if a part lost a hand-off, high: the launch's full 32-bit epoch}, so a
// word left by anything else never matches: a zeroed word has epoch 0 (never issued), an
// older launch's counter has an older epoch, and — the hand-off region being reused across
// batch layouts — an 8-byte hand-off granule that now sits where a counter lands carries
// its own launch's epoch in the same high half.  (Round 2 matched 24 epoch bits of a 4-byte
// word, which a granule's float half could match by chance.)  Returns the low word after
// this arrival.
__device__ unsigned split_arrive(uint64_t* c, unsigned epoch, bool lost) {
    uint64_t old = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        const unsigned cur = ((unsigned)(old >> 32) == epoch) ? (unsigned)old : 0u;
        const unsigned nw = ((cur & 0x7Fu) + 1u) | (cur & 0x80u) | (lost ? 0x80u : 0u);
        const uint64_t nv = ((uint64_t)epoch << 32) | nw;
        if (__hip_atomic_compare_exchange_strong(c, &old, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return nw;
    }
}


// Latency buckets (H) claim more than half of a CU's 160 KB LDS so that the dispatcher
// places one workgroup per CU: two 8-wave workgroups on one CU would share its SIMDs
// (4 waves per SIMD) while other CUs idle.

constexpr int kLatencyLdsFloats = 84 * 1024 / 4;

// Column-map LDS of the gather (large-vocabulary) instantiations.
template <int VS>
struct ColMapLds {
    static constexpr bool kOn = VS == kGatherVS;
    unsigned bm[kOn ? kMaxVocabWords : 1];
    int wpre[kOn ? kMaxVocabWords + 1 : 1];
    int cols[kOn ? kGatherVS : 1];
};

// Build the segment's column map when VS is the gather width; returns false (and the
// caller stops) when the segment uses more distinct columns than a compact row holds.
template <int VS>
__device__ __forceinline__ bool prepare_colmap(ColMapLds<VS>& m, ColMap& cm, const int32_t* tok, int N, int blank,
                                               int V) {
    cm.bm = m.bm;
    cm.wpre = m.wpre;
    cm.cols = m.cols;
    cm.n = 0;
    if (!ColMapLds<VS>::kOn) return true;
    cm.n = build_colmap(tok, N, blank, V, m.bm, m.wpre, m.cols);
    return cm.n <= kGatherVS;
}

// Row slots of the checkpointed walk (CkSrc), [kChunk][VS] each: two per walker wave (the next
// block's rows load while a block computes) where that keeps the LDS of a workgroup within its
// share at 4 waves per SIMD (VS == 32, and the one-wave kernels' two forward buffers), else one
// per walker wave (rows loaded at use, the next block's warmed into the L2).
// (One slot per walker wave everywhere measured slower in round 5.)
template <int VS, int W>
constexpr int kCkSlots = (W == 1 || VS == 32) ? 2 * W : W;

// Split kernels: waves per workgroup.  Beyond the W DP waves and the two helpers, the rest
// only keep the forward's barrier count and then walk speculative segments (walk_spec: more
// walkers, shorter segments).  177 VGPRs allow two waves per SIMD: 8 (12 waves = 168 VGPRs
// spilled 33 in the register-resident forward).  (6 waves, no extra walkers: config 2
// 51.4 -> 53.3 us in round 5.)
constexpr int kSplitWaves = 8;
constexpr int kQ0LdsFrames = 4096;  // Split::q0l rows (longer segments: fill_q0 after the walk)

template <int C, int VS, int W, int H, bool SP = false, int XW = 0>
__device__ __forceinline__ void align_dp_body(const AlignArgs& a) {
    // Checkpointed forward (MODE 2, CkSrc walk): the single-CU throughput kernels with two or
    // more waves (speculative walkers) and staged row widths; the one-wave (a lone walker would
    // recompute every block serially: slower than the bits it saves), latency (helper), split
    // and gathered-vocabulary kernels keep the bitmap.
    constexpr bool CK = !SP && H == 0 && VS != kGatherVS && W >= 2;
    constexpr bool WT = split_wt<C, VS, SP>();  // write-through hand-over of the bits to the last part
    // (CK: the walkers' row slots, one [32][VS] per wave, reuse the forward's buffers)
    constexpr int kLdsFloats = H ? (kLatencyLdsFloats > 4 * kChunk * VS ? kLatencyLdsFloats : 4 * kChunk * VS)
                                 : (CK ? kCkSlots<VS, W> : 2) * kChunk * VS;
    __shared__ float lds[kLdsFloats];
    __shared__ __attribute__((aligned(16))) float c0b[H || (CK && W >= 2) ? 2 * kChunk : 1];
    __shared__ __attribute__((aligned(16))) float xh[W > 1 ? 2 * W * kWave : 1];
    __shared__ unsigned cmask_lds[kMaxLdsFrames / kChunk + 1];
    __shared__ int tsb[3];
    __shared__ int blo_lds;  // walk_tail: the walk's lowest block (-1: no path)
    __shared__ int colrec_lds[W + H > 1 ? kMaxLdsFrames / kChunk + 1 : 1];  // walk_spec records
    __shared__ int sbuf_lds[3 * (W + H + XW)];
    __shared__ ColMapLds<VS> cml;
    __shared__ float xg_lds[SP && C == 1 ? 2 * 32 : 1];  // Split::xg
    __shared__ float q0_lds[SP && XW > 0 ? kQ0LdsFrames : 1];  // Split::q0l
    const int P = SP ? a.parts : 1;
    // Split grids: block b = ((s / 8) * P + p) * 8 + s % 8, so the parts of segment s share
    // b % 8 — one XCD under the observed round-robin dispatch — and read its emission rows
    // through one L2.  (Placement is a speed matter only; part p - 1 has the lower block
    // index either way, so it starts no later than part p.)  kArgXcdSpread (tests) puts part p
    // at b % 8 = (s + p) % 8 instead: every part of a segment on another XCD.
    const int part = SP ? ((int)blockIdx.x / kXcdStride) % P : 0;
    const int xslot = (int)blockIdx.x % kXcdStride;
    const int seg = SP ? ((int)blockIdx.x / kXcdStride / P) * kXcdStride +
                             ((a.flags & kArgXcdSpread) ? (xslot - part) & (kXcdStride - 1) : xslot)
                       : (int)blockIdx.x;
    if (SP && seg >= a.S) return;  // grid padded to a multiple of 8 segments
    const SegDesc d = load_desc(a.em_off, a.tok_off, a.blank_id, seg);
    const int want = (SP || a.parts > 1) ? launch_split_bucket(d.N, a.parts, a.split_id) : bucket_id(d.N, a.mode);
    if (want != (bucket_make(C, W, H ? 1 : 0) | (SP ? kSplitFlag : 0))) return;  // another instantiation owns it
    const int lane = (int)threadIdx.x;
    if (d.N <= 0 || d.T <= 0) {
        if (lane == 0 && part == 0) {
            a.t_start[seg] = 0;
            a.status[seg] = 1;
        }
        return;
    }
    ColMap cm;
    // More than kGatherVS distinct columns: the compact LDS row cannot hold the segment's
    // emissions, so one workgroup (part 0 of a split) runs the generic forward instead.
    const bool slow = !prepare_colmap(cml, cm, a.tok + d.tok0, d.N, d.blank, a.V);
    if (slow && part != 0) return;
    const float* E = a.em + d.row0 * a.V;
    unsigned* bits = a.bits + ((d.row0 >> 5) + seg) * (int64_t)a.bits_stride_cells;
    float* q0 = a.q0 + d.row0;
    float* cn = a.cn + ((d.row0 + kCnPad * (int64_t)seg) & ~(int64_t)3);
    double* c0acc = a.c0acc + ((d.row0 >> 5) + seg);
    WX_STAMP_RT(4);
    WX_STAMP(0);
    Split sp;
    if (SP) {
        sp.p = part;
        sp.P = P;
        sp.lanes = kWave * W * P;
        sp.tag = a.epoch;
        sp.xstride = (kMaxParts - 1) * kHaloCells;
        sp.spin = a.spin;
        uint64_t* xseg = a.xg + ((d.row0 >> 5) + seg) * (int64_t)sp.xstride;
        sp.xin = xseg + (part > 0 ? part - 1 : 0) * kHaloCells;
        sp.xout = xseg + part * kHaloCells;
        sp.xg = xg_lds;
        sp.q0l = (XW > 0 && d.T <= kQ0LdsFrames) ? q0_lds : nullptr;
    }
    if (SP && lane == 0) tsb[2] = 0;
    bool lost = false;
    if (!slow)
        lost = Forward<C, VS, CK ? 2 : 0, W, H != 0, SP, (H > 1 ? 2 : 1)>::run(
            d, E, a.V, a.tok, bits, q0, cn, nullptr, lds, c0b, xh, a.x4 != 0, cm, nullptr, &sp, c0acc);
    WX_STAMP(1);
    if (SP && lost) tsb[2] = 1;  // (any lane of the consumer or, register-resident kernels, the poller)
    wait_vm();
    block_fence();
    bool failed = false;
    if (SP && !slow) {  // release this part's bits / column-N history; the last part to arrive goes on
        if (lane == 0) {
            // (WT: every wave's stores drained above, then the barrier: no release)
            const bool fenced = !WT || (a.flags & kArgFenced);
            if (fenced) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                wait_vm();
            }
            const unsigned w = split_arrive(a.arrive + seg, a.epoch, tsb[2] != 0);
            tsb[0] = ((w & 0x7Fu) == (unsigned)P) ? 1 + (int)((w >> 7) & 1u) : 0;
            if (tsb[0]) {
                if (fenced) {  // (WT: the walk reads the parts' words with sc1 loads)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    wait_vm();
                }
                // every part has arrived: leave the counter clean for the next launch
                __hip_atomic_store(a.arrive + seg, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (tsb[0] == 0) {
            WX_STAMP(2);
            WX_STAMP(3);
            WX_STAMP_RT(5);
            return;
        }
        failed = tsb[0] == 2;
        __syncthreads();
    }
    const Layout lay = Layout::make(C, d.N, kWave * W * P);
    if (slow || failed) {
        // recovery: a lost hand-off (some part computed with a stale halo) or a segment whose
        // columns do not fit the compact row.  The whole workgroup recomputes the segment.
        if (!generic_forward(d.T, d.N, d.blank, E, a.V, a.tok + d.tok0, bits, lay, cn, q0, lds, kLdsFloats)) {
            if (lane == 0) {
                a.t_start[seg] = 0;
                a.status[seg] = slow ? 2 : 3;  // (N too large for the generic forward's LDS rows)
            }
            return;
        }
        wait_vm();
        block_fence();
    }
    int32_t* start = a.seg_start + d.tok0;
#ifdef WX_PHASE_TIMING
    WX_T(w0);
#endif
    // t_start, the walk and the change masks: several waves walk speculative segments, one per
    // wave (walk_spec, which also finds t_start); one wave walks alone
    const int nbw = ((d.T - 1) >> 5) + 1;
    const bool lds_walk = d.T <= kMaxLdsFrames;
    // q0 already in this workgroup's LDS (Split::q0l; the recovery paths write it to q0)
    const bool q0l_ok = SP && XW > 0 && d.T <= kQ0LdsFrames && !slow && !failed;
    const int K = lds_walk ? max(1, min(W + H + XW, nbw / kSpecMinBlocks)) : 1;
#ifdef WX_PHASE_TIMING
    WX_T(w1);
    unsigned long long wx_w2 = 0;
#endif
    auto walk_tail = [&](auto& wsrc) {
    int ts = 0, b_lo = -1;
    unsigned* cmask = lds_walk ? cmask_lds : a.cmask + ((d.row0 >> 5) + seg);
    if constexpr (W + H > 1) b_lo = walk_spec(wsrc, d.N, d.T, cn, cmask, lds_walk, K, colrec_lds, sbuf_lds, ts);
    if (lane < kWave) {  // wave 0: t_start, the walk, then the change masks -> start frames
        if constexpr (W + H == 1) {
            ts = column_argmax<WT>(cn, d.T);
            b_lo = walk_impl(wsrc, d.N, ts, cmask, lds_walk);
        }
        if (lane == 0) {
            a.t_start[seg] = ts;
            tsb[0] = ts;
        }
#ifdef WX_PHASE_TIMING
        WX_T(w2);
        wx_w2 = w2;
#endif
        if (!H && b_lo >= 0) {
            wave_fence();
            compact_starts(cmask, b_lo, (ts - 1) >> 5, start);
        }
        if (lane == 0) {
            tsb[1] = b_lo >= 0 ? 1 : 0;
            blo_lds = b_lo;
        }
    } else {
        if (H && !slow && !failed && !q0l_ok) fill_q0(E, a.V, d.T, q0, kWave);
    }
    if constexpr (H != 0) {  // latency / split kernels: the compaction over every wave
        block_fence();  // (wave 0's change masks, b_lo, t_start)
        const int bl = uniform(blo_lds);
        if (bl >= 0) compact_starts_par(cmask, bl, (uniform(tsb[0]) - 1) >> 5, start);
    }
#ifdef WX_PHASE_TIMING
    WX_T(w3);
    if (lane == 0 && blockIdx.x < 8192) {  // walk-phase split: argmax, walk, compaction
        unsigned long long* o = wx_loop + ((size_t)blockIdx.x * kLoopSlots + 15) * 3;
        o[0] = w1 - w0;
        o[1] = wx_w2 - w1;
        o[2] = w3 - wx_w2;
    }
#endif
    };
    if constexpr (CK) {
        CkSrc<C, VS> wsrc;
        wsrc.ck = reinterpret_cast<const float*>(bits);
        wsrc.lay = lay;
        wsrc.acc = c0acc;
        wsrc.E = E;
        wsrc.tok = a.tok + d.tok0;
        wsrc.T = d.T;
        wsrc.N = d.N;
        wsrc.V = a.V;
        wsrc.blank = d.blank;  // (as the forward reads it)
        wsrc.x4 = a.x4 != 0;
        // one-wave kernels: both forward buffers are the walker's two slots; else one per wave
        wsrc.slot[0] = lds + uniform((int)threadIdx.x >> 6) * kChunk * VS;
        wsrc.slot[1] = kCkSlots<VS, W> >= 2 * W ? wsrc.slot[0] + W * kChunk * VS : wsrc.slot[0];
        wsrc.junk = xh;  // (the forward's halo exchange, free now: 2 W 64 floats >= 1 KB when W > 1)
        walk_tail(wsrc);
    } else {
        BitSrc<C, WT> wsrc{bits, lay};
        walk_tail(wsrc);
    }
    wait_vm();
    block_fence();
    const int ts = tsb[0];
    const bool ok = tsb[1] != 0;
    WX_STAMP(2);
    // low bits: 0 aligned / 1 None; flags: which segments took the generic forward
    if (lane == 0) a.status[seg] = (ok ? 0 : 1) | (failed ? WX_STATUS_RECOVERED : 0) | (slow ? WX_STATUS_GENERIC : 0);
    if (!ok) return;
    // (staging costs one more round trip: it pays when every thread has several tokens)
    if (d.T + d.N <= kLdsFloats && d.N > 2 * (int)blockDim.x)
        merge_tokens_lds(E, a.V, a.tok + d.tok0, d.N, d.T, ts, q0l_ok ? q0_lds : q0, start, a.seg_end + d.tok0,
                         a.seg_score + d.tok0, lds);
    else
        merge_tokens(E, a.V, a.tok + d.tok0, d.N, ts, q0l_ok ? q0_lds : q0, start, a.seg_end + d.tok0,
                     a.seg_score + d.tok0);
    WX_STAMP(3);
    WX_STAMP_RT(5);
}

template <int C, int VS, int W, int H>
__global__ __launch_bounds__(kWave*(W + H)) __attribute__((amdgpu_waves_per_eu(H || VS == kGatherVS || C > 8 || W == 1 ? 1 : 4, H ? 2 : 8))) void align_dp_kernel(
    AlignArgs a) {
    align_dp_body<C, VS, W, H>(a);
}

// Split segments: P workgroups (parts, one per CU) per segment, grid = ceil(S / 8) * 8 * P.
template <int C, int VS, int W>
__global__ __launch_bounds__(kWave * kSplitWaves) __attribute__((amdgpu_waves_per_eu(1, 2))) void align_dp_split_kernel(
    AlignArgs a) {
    static_assert(W + 2 <= kSplitWaves && kSplitWaves <= 8, "split workgroup: W DP waves + 2 helpers + walkers");
    align_dp_body<C, VS, W, 2, true, kSplitWaves - W - 2>(a);
}

struct TrellisArgs {
    const float* em;
    const int64_t* em_off;
    int V;
    const int32_t* tok;
    const int64_t* tok_off;
    const int32_t* blank_id;
    float* tr;
    const int64_t* tr_off;
    int x4;
};

template <int C, int VS, int W>
__global__ __launch_bounds__(kWave * W) void trellis_kernel(TrellisArgs a) {
    __shared__ float lds[2 * kChunk * VS];
    __shared__ float xh[W > 1 ? 2 * W * kWave : 1];
    __shared__ ColMapLds<VS> cml;
    __shared__ __attribute__((aligned(16))) float rst[W * kWave * C];
    const int seg = blockIdx.x;
    const SegDesc d = load_desc(a.em_off, a.tok_off, a.blank_id, seg);
    if (bucket_id(d.N) != bucket_make(C, W, 0)) return;
    float* tr = a.tr + a.tr_off[seg];
    const int lane = (int)threadIdx.x;
    if (d.N == 0) {  // the whole single column is +inf (alignment.py:369-370 with num_tokens = 0)
        for (int t = lane; t <= d.T; t += kWave * W) tr[t] = INFINITY;
        return;
    }
    ColMap cm;
    if (!prepare_colmap(cml, cm, a.tok + d.tok0, d.N, d.blank, a.V)) {  // too many distinct columns
        const int64_t n = (int64_t)(d.T + 1) * (d.N + 1);
        for (int64_t i = lane; i < n; i += kWave * W) tr[i] = NAN;
        return;
    }
    const float* E = a.em + d.row0 * a.V;
    Forward<C, VS, 1, W, false>::run(d, E, a.V, a.tok, nullptr, nullptr, nullptr, tr, lds, nullptr, xh, a.x4 != 0,
                                     cm, rst);
}

// Development builds for A/B timing of V <= 32 batches (tools/ab): -DWX_DEV_V32 instantiates
// the V <= 32 kernels only (a third of the compile time); wider vocabularies are NOT served.
#ifdef WX_DEV_V32
#define WX_VS64 32
#define WX_VSG 32
#else
#define WX_VS64 64
#define WX_VSG kGatherVS
#endif

// Launchers of the kernel templates above.  Each instantiation is compiled in one of the
// shards of wx_align_inst.hip (explicit instantiations, built in parallel); the host ABI in
// wx_align.hip only references them.
template <int C, int VS, int W, int H>
void launch_align_dp(dim3 grid, hipStream_t s, const AlignArgs& a);
template <int C, int VS, int W>
void launch_align_split(dim3 grid, hipStream_t s, const AlignArgs& a);
template <int C, int VS, int W>
void launch_trellis(dim3 grid, hipStream_t s, const TrellisArgs& a);

}  // namespace wx

#endif  // WX_ALIGN_DP_H
