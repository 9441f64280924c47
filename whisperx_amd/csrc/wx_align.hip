// wx_align.hip — host C ABI of include/wx_align.h and the non-template kernels
// (materialised-trellis backtrack, merge_repeats, Binarize, VAD aggregation).  The fused DP
// and get_trellis kernel templates live in wx_align_dp.h; their instantiations are compiled
// in the shards of wx_align_inst.hip.
#include "wx_align_dp.h"
#ifdef WX_PHASE_TIMING  // one TU: the phase-timing device arrays must be a single copy
#include "wx_align_inst.hip"
#endif

namespace wx {

// ------------------------------------------------------------------------------------
// backtrack() from a materialised trellis: recompute the decision bits from the trellis
// (one column word per thread: 32 rows of one cell), argmax of column N, shared walk,
// then expand the per-token spans into the reference's Point list.
struct BacktrackArgs {
    const float* tr;
    const int64_t* tr_off;
    const float* em;
    const int64_t* em_off;
    int V;
    const int32_t* tok;
    const int64_t* tok_off;
    const int32_t* blank_id;
    int32_t* path_tok;
    int32_t* path_time;
    float* path_prob;
    int32_t* path_len;
    int32_t* t_start;
    unsigned* bits;
    int bits_stride_cells;
    int32_t* start;  // workspace: per-token start frames (CSR by tok_off)
    unsigned* cmask; // workspace: walk change masks
};

__global__ __launch_bounds__(256) void backtrack_kernel(BacktrackArgs a) {
    const int seg = blockIdx.x;
    const SegDesc d = load_desc(a.em_off, a.tok_off, a.blank_id, seg);
    const int T = d.T, N = d.N;
    const float* tr = a.tr + a.tr_off[seg];
    const float* E = a.em + d.row0 * a.V;
    const int32_t* tok = a.tok + d.tok0;
    const int64_t W = (int64_t)N + 1;
    const int cpl = max(1, (N + kWave - 1) / kWave);
    unsigned* bits = a.bits + ((d.row0 >> 5) + seg) * (int64_t)a.bits_stride_cells;
    const int nblk = (T + kChunk - 1) / kChunk;
    // (1) decision words: word (b, cell j) bit 31-s = changed>stayed at decision u = 32b+s
    const int nwords = nblk * cpl * kWave;
    for (int i = threadIdx.x; i < nwords; i += blockDim.x) {
        const int g = i % kWave;
        const int k = (i / kWave) % cpl;
        const int b = i / (kWave * cpl);
        const int j = g * cpl + k + 1;
        unsigned wv = 0u;
        if (j <= N) {
            int tk = tok[j - 1];
            tk = (tk >= 0 && tk < a.V) ? tk : 0;
            for (int s = 0; s < kChunk; ++s) {
                const int u = b * kChunk + s;
                unsigned bit = 0u;
                if (u < T) {
                    const float stayed = tr[(int64_t)u * W + j] + E[(int64_t)u * a.V + d.blank];
                    const float changed = tr[(int64_t)u * W + j - 1] + E[(int64_t)u * a.V + tk];
                    bit = changed > stayed ? 1u : 0u;
                }
                wv = (wv << 1) | bit;
            }
        }
        bits[((int64_t)b * cpl + k) * kWave + g] = wv;
    }
    // (2) argmax of column N over rows 0..T (first max, NaN counts as max)
    __shared__ float sv[256];
    __shared__ int si[256];
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    bool bn = false;
    for (int t = threadIdx.x; t <= T; t += blockDim.x) {
        const float v = tr[(int64_t)t * W + N];
        if (bn) continue;
        if (v != v) {
            bn = true;
            bv = v;
            bi = t;
        } else if (bi == 0x7fffffff || v > bv) {
            bv = v;
            bi = t;
        }
    }
    sv[threadIdx.x] = bn ? NAN : bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            const float v1 = sv[threadIdx.x], v2 = sv[threadIdx.x + off];
            const int i1 = si[threadIdx.x], i2 = si[threadIdx.x + off];
            const bool n1 = v1 != v1 && i1 != 0x7fffffff, n2 = v2 != v2 && i2 != 0x7fffffff;
            bool take2;
            if (i2 == 0x7fffffff) take2 = false;
            else if (i1 == 0x7fffffff) take2 = true;
            else if (n1 && n2) take2 = i2 < i1;
            else if (n1) take2 = false;
            else if (n2) take2 = true;
            else if (v2 > v1) take2 = true;
            else if (v1 > v2) take2 = false;
            else take2 = i2 < i1;
            if (take2) {
                sv[threadIdx.x] = v2;
                si[threadIdx.x] = i2;
            }
        }
        __syncthreads();
    }
    const int ts = (N == 0) ? 0 : si[0];
    if (threadIdx.x == 0) a.t_start[seg] = ts;
    __threadfence_block();
    __syncthreads();
    // (3) walk (wave 0)
    int32_t* start = a.start + d.tok0;
    __shared__ int ok_sh;
    if (threadIdx.x < kWave) {
        Layout lay;
        lay.C = cpl;
        lay.G = kWave;
        lay.n_short = 0;
        lay.lanes = kWave;
        unsigned* cmask = a.cmask + ((d.row0 >> 5) + seg);
        const int b_lo = walk<0>(bits, lay, N, ts, cmask, false);
        if (b_lo >= 0) {
            wave_fence();
            compact_starts(cmask, b_lo, (ts - 1) >> 5, start);
        }
        const bool ok = b_lo >= 0;
        if (threadIdx.x == 0) ok_sh = ok ? 1 : 0;
    }
    wait_vm();
    block_fence();
    const bool ok = ok_sh != 0;
    if (threadIdx.x == 0) a.path_len[seg] = ok ? (ts - start[0]) : -1;
    if (!ok) return;
    // (4) expand spans -> Points (forward order) at path offset em_off[seg]
    const int base_t = start[0];
    int32_t* ptok = a.path_tok + d.row0;
    int32_t* ptime = a.path_time + d.row0;
    float* pprob = a.path_prob + d.row0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const int s = start[k];
        const int e = (k + 1 < N) ? start[k + 1] : ts;
        int tk = tok[k];
        tk = (tk >= 0 && tk < a.V) ? tk : 0;
        for (int x = s; x < e; ++x) {
            ptok[x - base_t] = k;
            ptime[x - base_t] = x;
            pprob[x - base_t] = exp_cr(E[(int64_t)x * a.V + (x == s ? tk : 0)]);
        }
    }
}

// ------------------------------------------------------------------------------------
// merge_repeats over arbitrary paths: run boundaries by ballot, then one fp64 left-to-right
// sum per run.  One wave per path.
struct MergeArgs {
    const int32_t* ptok;
    const int32_t* ptime;
    const float* pprob;
    const int64_t* path_off;
    const int32_t* path_len;
    int32_t* seg_tok;
    int32_t* seg_start;
    int32_t* seg_end;
    double* seg_score;
    int32_t* seg_count;
};

__global__ __launch_bounds__(kWave) void merge_repeats_kernel(MergeArgs a) {
    const int seg = blockIdx.x;
    const int lane = lane_id();
    const int L = uniform(a.path_len[seg]);
    if (L <= 0) {
        if (lane == 0) a.seg_count[seg] = 0;
        return;
    }
    const int64_t off = a.path_off[seg];
    const int32_t* pt = a.ptok + off;
    const int32_t* pm = a.ptime + off;
    const float* pp = a.pprob + off;
    int32_t* gstart = a.seg_end + off;  // scratch: run start indices, overwritten below
    int G = 0;
    for (int i0 = 0; i0 < L; i0 += kWave) {
        const int i = i0 + lane;
        bool flag = false;
        if (i < L) flag = (i == 0) || (pt[i] != pt[i - 1]);
        const unsigned long long m = __ballot(flag);
        const int pos = G + __popcll(m & ((1ull << lane) - 1ull));
        if (flag) gstart[pos] = i;
        G += __popcll(m);
    }
    wait_vm();
    block_fence();
    for (int g0 = 0; g0 < G; g0 += kWave) {
        const int g = g0 + lane;
        int i1 = 0, i2 = 0;
        if (g < G) {
            i1 = gstart[g];
            i2 = (g + 1 < G) ? gstart[g + 1] : L;
        }
        wait_vm();
        block_fence();
        if (g < G) {
            double sum = 0.0;
            for (int i = i1; i < i2; ++i) sum += (double)pp[i];
            a.seg_tok[off + g] = pt[i1];
            a.seg_start[off + g] = pm[i1];
            a.seg_end[off + g] = pm[i2 - 1] + 1;
            a.seg_score[off + g] = sum / (double)(i2 - i1);
        }
        wait_vm();
        block_fence();
    }
    if (lane == 0) a.seg_count[seg] = G;
}

// ------------------------------------------------------------------------------------
// Binarize (vad.py:118-180), one wave per score column.  Event driven: the wave scans 256
// frames per iteration for the next transition (ballot + ffs) instead of stepping the FSM
// frame by frame; a min-cut split takes a wave argmin over the second half of the current
// score list.  The score list is [stale?] + frames [lo, i): the reference keeps one stale
// element (the deactivation frame, or frame 0) in front of the frames appended while active.
struct BinarizeArgs {
    const float* y;
    const int64_t* f_off;
    const double* sw_start;
    const double* sw_step;
    const double* sw_dur;
    float onset, offset;
    double maxd, pad_on, pad_off;
    double* rs;
    double* re;
    const int64_t* reg_off;
    int64_t* reg_count;
};

__device__ __forceinline__ double sw_mid(double st, double step, double dur, int64_t i) {
    const double s = st + (double)i * step;
    const double e = s + dur;
    return 0.5 * (s + e);
}

// (value, frame) argmin with the reference's np.argmin semantics over increasing frames:
// first NaN wins, else the first minimum.
__device__ __forceinline__ void argmin_combine(float& v, int64_t& f, bool& nan, float v2, int64_t f2, bool nan2) {
    if (f2 < 0) return;
    if (f < 0) {
        v = v2; f = f2; nan = nan2;
        return;
    }
    bool take;
    if (nan && nan2) take = f2 < f;
    else if (nan) take = false;
    else if (nan2) take = true;
    else if (v2 < v) take = true;
    else if (v < v2) take = false;
    else take = f2 < f;
    if (take) {
        v = v2; f = f2; nan = nan2;
    }
}

// Region output of a Binarize wave: region n is held by lane n % 64 and the wave writes 64
// at a time (one coalesced store per array).  A store per region made every later load of
// the wave wait for the store's acknowledgement (vmcnt counts both, in order): ~0.5 us per
// region on dense scores.
struct RegionOut {
    double* rs;
    double* re;
    int64_t cap;
    int64_t n = 0;
    bool overflow = false;
    double bs = 0.0, be = 0.0;
    __device__ __forceinline__ void emit(double s, double e, int lane) {
        if (!((e - s) > 1e-6)) return;  // pyannote Segment truthiness: empty segments are not stored
        if (n >= cap) {
            overflow = true;
            return;
        }
        if (lane == (int)(n & (kWave - 1))) {
            bs = s;
            be = e;
        }
        ++n;
        if ((n & (kWave - 1)) == 0) {
            rs[n - kWave + lane] = bs;
            re[n - kWave + lane] = be;
        }
    }
    __device__ __forceinline__ void flush(int lane) {
        const int r = (int)(n & (kWave - 1));
        if (lane < r) {
            rs[n - r + lane] = bs;
            re[n - r + lane] = be;
        }
    }
};

#ifndef WX_SCANQ
#define WX_SCANQ 2
#endif
constexpr int kScanQ = WX_SCANQ;  // frames per lane per event-scan iteration (1 h merge_chunks A/B: 2 -> 7.8 ms, 4 -> 9.4, 8 -> 12.7)

__global__ __launch_bounds__(kWave) void binarize_kernel(BinarizeArgs a) {
    const int file = blockIdx.x;
    const int lane = lane_id();
    const int64_t f0 = a.f_off[file];
    const int64_t F = a.f_off[file + 1] - f0;
    const float* y = a.y + f0;
    const double st = a.sw_start[file], step = a.sw_step[file], dur = a.sw_dur[file];
    const int64_t r0 = a.reg_off[file];
    const int64_t cap = a.reg_off[file + 1] - r0;
    double* rs = a.rs + r0;
    double* re = a.re + r0;
    RegionOut out{rs, re, cap};
    auto emit = [&](double s, double e) { out.emit(s, e, lane); };
    if (F <= 0) {
        if (lane == 0) a.reg_count[file] = 0;
        return;
    }
    double start = sw_mid(st, step, dur, 0);
    bool active = y[0] > a.onset;
    bool has_stale = !active;  // curr = [0]: stale when inactive, else the range [0, 1)
    int64_t stale = 0;
    int64_t lo = active ? 0 : 1;
    int64_t i = 1;
    while (i < F) {
        // ---- find the next event frame e >= i
        int64_t ev = -1;
        bool split = false;
        for (int64_t base = i; base < F && ev < 0; base += kScanQ * kWave) {
            unsigned long long m[kScanQ];
            unsigned long long ms[kScanQ];
#pragma unroll
            for (int q = 0; q < kScanQ; ++q) {
                const int64_t f = base + q * kWave + lane;
                bool p = false, ps = false;
                if (f < F) {
                    const float v = y[f];
                    if (!active) {
                        p = v > a.onset;
                    } else {
                        ps = (sw_mid(st, step, dur, f) - start) > a.maxd;
                        p = ps || (v < a.offset);
                    }
                }
                m[q] = __ballot(p);
                ms[q] = __ballot(ps);
            }
#pragma unroll
            for (int q = 0; q < kScanQ; ++q) {
                if (ev < 0 && m[q]) {
                    const int l = __ffsll((long long)m[q]) - 1;
                    ev = base + q * kWave + l;
                    split = (ms[q] >> l) & 1ull;
                }
            }
        }
        if (ev < 0) break;
        const double tev = sw_mid(st, step, dur, ev);
        if (!active) {
            start = tev;
            active = true;
            lo = ev + 1;  // the activation frame itself is not appended (vad.py:171-175)
            i = ev + 1;
            continue;
        }
        if (split) {
            // curr = [stale?] + frames [lo, ev); search positions [len/2, len)
            const int64_t len = (has_stale ? 1 : 0) + (ev - lo);
            const int64_t sa = len / 2;
            float bv = 0.f;
            int64_t bf = -1;
            bool bn = false;
            const int64_t fa = lo + max<int64_t>(sa - (has_stale ? 1 : 0), 0);
            for (int64_t f0 = fa + lane; f0 < ev; f0 += 8 * kWave) {  // 8 loads in flight per lane
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int64_t f = f0 + u * kWave;
                    v[u] = f < ev ? y[f] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {  // this lane's frames in increasing order
                    const int64_t f = f0 + u * kWave;
                    if (f < ev) argmin_combine(bv, bf, bn, v[u], f, v[u] != v[u]);
                }
            }
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const float v2 = __shfl_xor(bv, off);
                const int64_t f2 = __shfl_xor(bf, off);
                const bool n2 = __shfl_xor((int)bn, off) != 0;
                argmin_combine(bv, bf, bn, v2, f2, n2);
            }
            int64_t cut = bf;
            bool cut_is_stale = false;
            if (has_stale && sa == 0) {  // position 0 (the stale element) is a candidate and comes first
                const float sv = y[stale];
                const bool sn = sv != sv;
                if (bf < 0 || sn || (!bn && !(bv < sv))) {
                    cut = stale;
                    cut_is_stale = true;
                }
            }
            const double mt = sw_mid(st, step, dur, cut);
            emit(start - a.pad_on, mt + a.pad_off);
            start = mt;
            if (!cut_is_stale) lo = cut + 1;
            has_stale = false;
            i = ev + 1;  // frame ev appended: range becomes [lo, ev+1)
        } else {
            emit(start - a.pad_on, tev + a.pad_off);
            start = tev;
            active = false;
            has_stale = true;
            stale = ev;
            i = ev + 1;
        }
    }
    if (active) {
        const double tl = (F == 1) ? sw_mid(st, step, dur, 0) : sw_mid(st, step, dur, F - 1);
        emit(start - a.pad_on, tl + a.pad_off);
    }
    out.flush(lane);
    if (lane == 0) a.reg_count[file] = out.overflow ? -1 : out.n;
}

// ------------------------------------------------------------------------------------
// Binarize, two-pass form (wx_binarize_ex).  Pass 1 (binarize_words_kernel: one thread per
// 64-frame block of every file, chip-wide) writes the block's onset word (bit k: y > onset),
// offset word (bit k: y < offset) and first-minimum record (np.argmin order: the first NaN,
// else the first smallest value).  Pass 2 (binarize_fsm_kernel: one wave per file) runs the
// state machine event to event: the next activation / deactivation is the next set bit of
// a word array, found in a window of 64 words (4096 frames) held one word per lane with the
// following window prefetched; the first frame past max_duration comes from the window
// geometry; a min-cut is the argmin over the records of the full blocks in its range and
// the frames of the two partial blocks at its ends.  Cost per event is a few dozen wave
// instructions, independent of the gap to the next event.  Block b of a file starting at
// frame f0 is word (f0 >> 6) + file + b.
struct BinWords {
    unsigned long long* on;   // y > onset
    unsigned long long* off;  // y < offset
    float* mv;                // block minimum (NaN when the block holds one: the first)
    int32_t* mi;              // its file-local frame; -1 for words past the file's end
};

__host__ __device__ inline int64_t bin_word_base(int64_t f0, int file) { return (f0 >> 6) + file; }
inline int64_t bin_words(int64_t total_frames, int n_files) { return (total_frames >> 6) + n_files + 1; }

struct BinWordArgs {
    const float* y;
    const int64_t* f_off;
    int n_files;
    int64_t n_words;
    float onset, offset;
    BinWords w;
};

// One wave per 64 words: the wave loads each word's 64 frames in one coalesced instruction
// (lane = frame) into a padded LDS tile, then every lane scans its own word's column.  (A
// lane reading its own 64 frames touched 64 cache lines per load instruction: 16 us per
// hour against ~3 us.)
__global__ __launch_bounds__(kWave) void binarize_words_kernel(BinWordArgs a) {
    __shared__ float tile[kWave * (kWave + 1)];
    const int lane = lane_id();
    const int64_t g = (int64_t)blockIdx.x * kWave + lane;
    int64_t gf = 0, fb = -1;  // this lane's word: first frame (global) and file-local
    int n = 0;                // frames in it
    if (g < a.n_words) {
        int lo = 0, hi = a.n_files - 1;  // the last file whose first word is <= g
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (bin_word_base(a.f_off[mid], mid) <= g) lo = mid;
            else hi = mid - 1;
        }
        const int64_t f0 = a.f_off[lo];
        const int64_t F = a.f_off[lo + 1] - f0;
        fb = (g - bin_word_base(f0, lo)) << 6;
        if (fb < F) {
            n = (int)min<int64_t>(kWave, F - fb);
            gf = f0 + fb;
        }
    }
    {
        float v[kWave];  // all 64 loads in flight before the first wait
#pragma unroll
        for (int r = 0; r < kWave; ++r) {
            const int64_t gr = (int64_t)readlane64((unsigned long long)gf, r);
            const int nr = __builtin_amdgcn_readlane(n, r);
            v[r] = a.y[gr + min(lane, max(nr - 1, 0))];
        }
#pragma unroll
        for (int r = 0; r < kWave; ++r) tile[r * (kWave + 1) + lane] = v[r];
    }
    __syncthreads();
    unsigned long long on = 0, off = 0;
    float mv = 0.f;
    int32_t mi = -1;
    if (n > 0) {
        bool nan = false;
        // a uniform trip count with a per-lane predicate and selects: a loop whose exit is
        // divergent let the compiler keep the (uniform) index of the last update in an SGPR
#pragma unroll 8
        for (int k = 0; k < kWave; ++k) {
            const float v = tile[lane * (kWave + 1) + k];
            const bool in = k < n;
            on |= (unsigned long long)(in && v > a.onset) << k;
            off |= (unsigned long long)(in && v < a.offset) << k;
            const bool vn = v != v;
            const bool take = in && (mi < 0 || (!nan && (vn || v < mv)));
            mv = take ? v : mv;
            mi = take ? k : mi;
            nan = take ? vn : nan;
        }
        mi += (int32_t)fb;
        // frame 0 decides the initial state either way (vad.py:142): mark it a reset when it
        // does not activate (the state machines never search the offset word at frame 0)
        if (fb == 0 && !(on & 1ull)) off |= 1ull;
    }
    if (g < a.n_words) {
        a.w.on[g] = on;
        a.w.off[g] = off;
        a.w.mv[g] = mv;
        a.w.mi[g] = mi;
    }
}

struct BinWin {  // words [base, base + 64) one per lane, and the next 64 prefetched
    int64_t base;
    unsigned long long w, nx;
};

__device__ __forceinline__ unsigned long long bin_ld(const unsigned long long* p, int64_t i, int64_t nw) {
    return i < nw ? p[i] : 0ull;
}

// First frame >= from whose bit is set in p[0, nw), or -1.
__device__ __forceinline__ int64_t bin_next(const unsigned long long* p, int64_t nw, BinWin& s, int64_t from,
                                            int lane) {
    int64_t wi = uniform64(from >> 6);
    unsigned long long low = ~0ull << (from & 63);
    while (wi < nw) {
        s.base = uniform64(s.base);
        if (wi >= s.base + kWave && wi < s.base + 2 * kWave) {
            s.base += kWave;
            s.w = s.nx;
            s.nx = bin_ld(p, s.base + kWave + lane, nw);
        } else if (wi < s.base || wi >= s.base + kWave) {
            s.base = wi;
            s.w = bin_ld(p, wi + lane, nw);
            s.nx = bin_ld(p, wi + kWave + lane, nw);
        }
        const int k = (int)(wi - s.base);
        unsigned long long x = s.w;
        if (lane == k) x &= low;
        const unsigned long long m = __ballot(lane >= k && x != 0ull);
        if (m) {  // results made wave-uniform: the state machine around this runs as scalar code
            const int l = __ffsll((long long)m) - 1;
            const unsigned long long xw = readlane64(x, l);
            return uniform64(((s.base + l) << 6) + (__ffsll((long long)xw) - 1));
        }
        wi = uniform64(s.base + kWave);
        low = ~0ull;
    }
    return -1;
}

// np.argmin order over frames [fa, ev) (fa < ev) from the block records and the partial blocks.
__device__ __forceinline__ void bin_argmin(const float* y, const float* mv, const int32_t* mi, int64_t fa,
                                           int64_t ev, int lane, float& bv, int64_t& bf, bool& bn) {
    bv = 0.f;
    bf = -1;
    bn = false;
    const int64_t b0 = (fa + 63) >> 6, b1 = ev >> 6;
    if (b0 >= b1) {  // no full block: at most 127 frames
        for (int64_t f = fa + lane; f < ev; f += kWave) {
            const float v = y[f];
            argmin_combine(bv, bf, bn, v, f, v != v);
        }
    } else {
        const int64_t fh = fa + lane, ft = (b1 << 6) + lane;
        const float vh = fh < (b0 << 6) ? y[fh] : 0.f;
        const float vt = ft < ev ? y[ft] : 0.f;
        for (int64_t b = b0 + lane; b < b1; b += kWave) {
            const float v = mv[b];
            argmin_combine(bv, bf, bn, v, (int64_t)mi[b], v != v);
        }
        if (fh < (b0 << 6)) argmin_combine(bv, bf, bn, vh, fh, vh != vh);
        if (ft < ev) argmin_combine(bv, bf, bn, vt, ft, vt != vt);
    }
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const float v2 = __shfl_xor(bv, off);
        const int64_t f2 = __shfl_xor(bf, off);
        const bool n2 = __shfl_xor((int)bn, off) != 0;
        argmin_combine(bv, bf, bn, v2, f2, n2);
    }
    bv = uniformf(bv);
    bf = uniform64(bf);
    bn = uniform((int)bn) != 0;
}

__global__ __launch_bounds__(kWave) void binarize_fsm_kernel(BinarizeArgs a, BinWords w) {
    const int file = blockIdx.x;
    const int lane = lane_id();
    const int64_t f0 = a.f_off[file];
    const int64_t F = a.f_off[file + 1] - f0;
    const float* y = a.y + f0;
    const double st = a.sw_start[file], step = a.sw_step[file], dur = a.sw_dur[file];
    const int64_t r0 = a.reg_off[file];
    const int64_t cap = a.reg_off[file + 1] - r0;
    double* rs = a.rs + r0;
    double* re = a.re + r0;
    const int64_t wb = bin_word_base(f0, file), nw = (F + 63) >> 6;
    const unsigned long long* won = w.on + wb;
    const unsigned long long* woff = w.off + wb;
    RegionOut out{rs, re, cap};
    auto emit = [&](double s, double e) { out.emit(s, e, lane); };
    if (F <= 0) {
        if (lane == 0) a.reg_count[file] = 0;
        return;
    }
    BinWin son{-(1ll << 40), 0ull, 0ull}, soff{-(1ll << 40), 0ull, 0ull};
    double start = sw_mid(st, step, dur, 0);
    // the split rule at frame f: mid(f) - start > max_duration; non-decreasing in f
    auto past = [&](int64_t f) { return (sw_mid(st, step, dur, f) - start) > a.maxd; };
    bool active = uniformf(y[0]) > a.onset;
    bool has_stale = !active;  // curr = [0]: stale when inactive, else the range [0, 1)
    int64_t stale = 0;
    int64_t lo = active ? 0 : 1;
    int64_t i = 1;
    while (i < F) {
        i = uniform64(i);
        lo = uniform64(lo);
        if (!active) {
            const int64_t ev = bin_next(won, nw, son, i, lane);
            if (ev < 0) break;
            start = sw_mid(st, step, dur, ev);
            active = true;
            lo = ev + 1;  // the activation frame itself is not appended (vad.py:171-175)
            i = ev + 1;
            continue;
        }
        int64_t fd = bin_next(woff, nw, soff, i, lane);  // next deactivation frame
        const int64_t last = fd < 0 ? F - 1 : fd;
        if (!past(last)) {  // no split before the deactivation (the split rule is checked first)
            if (fd < 0) break;
            const double tev = sw_mid(st, step, dur, fd);
            emit(start - a.pad_on, tev + a.pad_off);
            start = tev;
            active = false;
            has_stale = true;
            stale = fd;
            i = fd + 1;
            continue;
        }
        // first frame in [i, last] past max_duration: estimate from the geometry, then settle
        const double x = (start + a.maxd - st - 0.5 * dur) / step;
        int64_t ev = (x > (double)i) ? (x < (double)last ? (int64_t)x : last) : i;
        while (ev > i && past(ev - 1)) --ev;
        while (!past(ev)) ++ev;
        // curr = [stale?] + frames [lo, ev); min-cut over positions [len/2, len)
        const int64_t len = (has_stale ? 1 : 0) + (ev - lo);
        const int64_t sa = len / 2;
        const int64_t fa = lo + max<int64_t>(sa - (has_stale ? 1 : 0), 0);
        float bv = 0.f;
        int64_t bf = -1;
        bool bn = false;
        if (fa < ev) bin_argmin(y, w.mv + wb, w.mi + wb, fa, ev, lane, bv, bf, bn);
        int64_t cut = bf;
        bool cut_is_stale = false;
        if (has_stale && sa == 0) {  // position 0 (the stale element) is a candidate and comes first
            const float sv = uniformf(y[stale]);
            const bool sn = sv != sv;
            if (bf < 0 || sn || (!bn && !(bv < sv))) {
                cut = stale;
                cut_is_stale = true;
            }
        }
        const double mt = sw_mid(st, step, dur, cut);
        emit(start - a.pad_on, mt + a.pad_off);
        start = mt;
        if (!cut_is_stale) lo = cut + 1;
        has_stale = false;
        i = ev + 1;  // frame ev appended: range becomes [lo, ev+1)
    }
    if (active) {
        const double tl = (F == 1) ? sw_mid(st, step, dur, 0) : sw_mid(st, step, dur, F - 1);
        emit(start - a.pad_on, tl + a.pad_off);
    }
    out.flush(lane);
    if (lane == 0) a.reg_count[file] = out.overflow ? -1 : out.n;
}

// ------------------------------------------------------------------------------------
// Binarize as a parallel scan (wx_binarize_ex when offset <= onset, the reference's
// defaults and every whisperX call).  Without the max_duration rule the hysteresis state
// after frame f is that of the last decisive frame <= f (y > onset: 1, y < offset: 0; no
// frame is both when offset <= onset), so a 64-frame block's state word follows from its
// onset / offset words and the state before it by one carry-propagate addition, and a
// block's transfer function (state after it, per state before it) composes associatively.
// binarize_scan_kernel (one 1024-thread workgroup per file) scans the blocks' transfer
// functions, derives every block's activation (0 -> 1) and deactivation (1 -> 0) words and
// scatters their frames, in order, into per-file region lists: region k runs from
// activation a_k to deactivation d_k.  Wave 0 then takes the regions 64 at a time, one per
// lane: a region that never exceeds max_duration (mid(d_k) - mid(a_k) <= max_duration; the
// rule's predicate is non-decreasing in the frame) is emitted as it is.  The first one that
// does runs the sequential active-state machine with min-cuts (bin_active_run) from a_k
// until a deactivation that no split overrides: a split at a deactivation frame keeps the
// region active (vad.py:150-161, `if ... elif`), so that machine may absorb the following
// regions; the batch resumes at the first region activated after its end, where the real
// and the scanned state agree again (a deactivation frame resets both).
struct BinFile {
    const float* y;
    int64_t F;
    double st, step, dur;
    const unsigned long long* zw;  // offset words (frame 0's bit: a reset when it does not activate)
    int64_t nw;
    const float* mv;
    const int32_t* mi;
};

// Active from frame i on (score list [stale?] + frames [lo, i), region start `start`) until
// the first deactivation no split overrides (returned) or the file's end (-1, final region
// emitted with the last frame's time, vad.py:178-180).
__device__ int64_t bin_active_run(const BinarizeArgs& a, const BinFile& f, double start, bool has_stale,
                                  int64_t stale, int64_t lo, int64_t i, RegionOut& out, int lane) {
    BinWin soff{-(1ll << 40), 0ull, 0ull};
    auto past = [&](int64_t fr) { return (sw_mid(f.st, f.step, f.dur, fr) - start) > a.maxd; };
    while (true) {
        i = uniform64(i);
        lo = uniform64(lo);
        if (i >= f.F) {
            out.emit(start - a.pad_on, sw_mid(f.st, f.step, f.dur, f.F - 1) + a.pad_off, lane);
            return -1;
        }
        const int64_t fd = bin_next(f.zw, f.nw, soff, i, lane);
        const int64_t last = fd < 0 ? f.F - 1 : fd;
        if (!past(last)) {
            out.emit(start - a.pad_on, sw_mid(f.st, f.step, f.dur, last) + a.pad_off, lane);
            return fd;
        }
        const double x = (start + a.maxd - f.st - 0.5 * f.dur) / f.step;
        int64_t ev = (x > (double)i) ? (x < (double)last ? (int64_t)x : last) : i;
        while (ev > i && past(ev - 1)) --ev;
        while (!past(ev)) ++ev;
        const int64_t len = (has_stale ? 1 : 0) + (ev - lo);
        const int64_t sa = len / 2;
        const int64_t fa = lo + max<int64_t>(sa - (has_stale ? 1 : 0), 0);
        float bv = 0.f;
        int64_t bf = -1;
        bool bn = false;
        if (fa < ev) bin_argmin(f.y, f.mv, f.mi, fa, ev, lane, bv, bf, bn);
        int64_t cut = bf;
        bool cut_is_stale = false;
        if (has_stale && sa == 0) {
            const float sv = uniformf(f.y[stale]);
            const bool sn = sv != sv;
            if (bf < 0 || sn || (!bn && !(bv < sv))) {
                cut = stale;
                cut_is_stale = true;
            }
        }
        const double mt = sw_mid(f.st, f.step, f.dur, cut);
        out.emit(start - a.pad_on, mt + a.pad_off, lane);
        start = mt;
        if (!cut_is_stale) lo = cut + 1;
        has_stale = false;
        i = ev + 1;
    }
}

// State word of a block (bit k: state after frame k) from its onset word G, offset word Z
// (disjoint) and the state before it: a carry generated at a G bit ripples up through the
// keep bits and is absorbed at a Z bit.
__device__ __forceinline__ unsigned long long bin_state_word(unsigned long long G, unsigned long long Z,
                                                             unsigned s_in) {
    const unsigned long long P = ~(G | Z);
    const unsigned long long A = G | P;
    return G | (P & ((A + G + (unsigned long long)s_in) ^ A ^ G));
}

// transfer functions as 2 bits (f(0) | f(1) << 1); "f then g"
__device__ __forceinline__ unsigned tf_then(unsigned f, unsigned g) {
    return ((g >> (f & 1u)) & 1u) | (((g >> ((f >> 1) & 1u)) & 1u) << 1);
}

constexpr int kBinWG = 1024;
// Wave 0's regions are staged in an LDS ring and written out 2048 at a time: a store per
// batch made the next batch's (prefetched) list loads wait for the stores too (vmcnt
// counts both, in order).
constexpr int kBinRing = 2048;
constexpr int kBinChunk = 8;  // per-thread loads issued together in the scan kernel's passes

// Exclusive scan over the workgroup in thread order ("a then b"), and the total.
template <class T, class Op>
__device__ __forceinline__ T wg_exclusive_scan(T x, T identity, Op op, T* lds, T& total) {
    const int lane = lane_id(), wv = threadIdx.x / kWave;
    T inc = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const T y = __shfl_up(inc, d);
        if (lane >= d) inc = op(y, inc);
    }
    if (lane == kWave - 1) lds[wv] = inc;
    __syncthreads();
    T pre = identity, tot = identity;
    for (int w = 0; w < kBinWG / kWave; ++w) {
        const T v = lds[w];
        if (w < wv) pre = op(pre, v);
        tot = op(tot, v);
    }
    total = tot;
    T ex = __shfl_up(inc, 1);
    if (lane == 0) ex = identity;
    __syncthreads();
    return op(pre, ex);
}

struct BinScanArgs {
    BinarizeArgs a;
    BinWords w;
    int32_t* ra;  // activation frames, file at f_off[file] + file (capacity F + 1)
    int32_t* rd;  // deactivation frames, same layout
};

__global__ __launch_bounds__(kBinWG) void binarize_scan_kernel(BinScanArgs sa) {
    __shared__ unsigned s_f[kBinWG / kWave];
    __shared__ unsigned long long s_n[kBinWG / kWave];
    __shared__ double s_rs[kBinRing], s_re[kBinRing];
    const BinarizeArgs& a = sa.a;
    const int file = blockIdx.x;
    const int t = threadIdx.x;
    const int lane = lane_id();
    const int64_t f0 = a.f_off[file];
    const int64_t F = a.f_off[file + 1] - f0;
    if (F <= 0) {
        if (t == 0) a.reg_count[file] = 0;
        return;
    }
    const int64_t nb = (F + 63) >> 6, wb = bin_word_base(f0, file);
    const unsigned long long* G = sa.w.on + wb;
    const unsigned long long* Z = sa.w.off + wb;
    int32_t* ra = sa.ra + f0 + file;
    int32_t* rd = sa.rd + f0 + file;
    const int64_t per = (nb + kBinWG - 1) / kBinWG;
    const int64_t b0 = min<int64_t>((int64_t)t * per, nb), b1 = min<int64_t>(b0 + per, nb);
    // pass 1: this thread's blocks as a transfer function, and their transition counts for
    // either state before them
    unsigned s[2] = {0u, 1u};
    unsigned long long cnt[2] = {0ull, 0ull};  // activations << 32 | deactivations
    for (int64_t bc = b0; bc < b1; bc += kBinChunk) {  // loads of a chunk issued together
        unsigned long long gv[kBinChunk], zv[kBinChunk];
#pragma unroll
        for (int j = 0; j < kBinChunk; ++j) {
            const int64_t b = min<int64_t>(bc + j, b1 - 1);
            gv[j] = G[b];
            zv[j] = Z[b];
        }
#pragma unroll
        for (int j = 0; j < kBinChunk; ++j) {
            if (bc + j >= b1) break;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const unsigned long long S = bin_state_word(gv[j], zv[j], s[q]);
                const unsigned long long prev = (S << 1) | s[q];
                cnt[q] += ((unsigned long long)__popcll(S & ~prev) << 32) | (unsigned long long)__popcll(prev & ~S);
                s[q] = (unsigned)(S >> 63);
            }
        }
    }
    unsigned ftot;
    const unsigned fpre = wg_exclusive_scan(s[0] | (s[1] << 1), 2u, tf_then, s_f, ftot);
    const unsigned s_in = fpre & 1u;  // inactive before frame 0
    unsigned long long ntot;
    const unsigned long long base =
        wg_exclusive_scan(cnt[s_in], 0ull, [](unsigned long long x, unsigned long long y) { return x + y; }, s_n, ntot);
    // pass 2: scatter the transition frames in order
    int64_t ia = (int64_t)(base >> 32), id = (int64_t)(base & 0xffffffffull);
    unsigned sv = s_in;
    for (int64_t bc = b0; bc < b1; bc += kBinChunk) {
        unsigned long long gv[kBinChunk], zv[kBinChunk];
#pragma unroll
        for (int j = 0; j < kBinChunk; ++j) {
            const int64_t b = min<int64_t>(bc + j, b1 - 1);
            gv[j] = G[b];
            zv[j] = Z[b];
        }
        for (int j = 0; j < kBinChunk && bc + j < b1; ++j) {
            const int64_t b = bc + j;
            const unsigned long long S = bin_state_word(gv[j], zv[j], sv);
            const unsigned long long prev = (S << 1) | sv;
            unsigned long long act = S & ~prev, deact = prev & ~S;
            while (act) {
                ra[ia++] = (int32_t)((b << 6) + __ffsll((long long)act) - 1);
                act &= act - 1;
            }
            while (deact) {
                rd[id++] = (int32_t)((b << 6) + __ffsll((long long)deact) - 1);
                deact &= deact - 1;
            }
            sv = (unsigned)(S >> 63);
        }
    }
    __syncthreads();  // the lists are complete (workgroup-scope release/acquire)
    const int64_t R = (int64_t)(ntot >> 32), ND = (int64_t)(ntot & 0xffffffffull);
    const int64_t r0 = a.reg_off[file];
    const int64_t cap = a.reg_off[file + 1] - r0;
    double* rs = a.rs + r0;
    double* re = a.re + r0;
    BinFile f;
    f.y = a.y + f0;
    f.F = F;
    f.st = a.sw_start[file];
    f.step = a.sw_step[file];
    f.dur = a.sw_dur[file];
    // ---- no region exceeds max_duration (checked by all threads): every region is emitted as
    // it is, at the position a workgroup prefix sum gives it
    {
        const int64_t perR = (R + kBinWG - 1) / kBinWG;
        const int64_t k0 = min<int64_t>((int64_t)t * perR, R), k1 = min<int64_t>(k0 + perR, R);
        auto region = [&](int64_t kk, int32_t av, int32_t dv, double& s, double& e) {  // 0 empty, 1 emitted, 2 long
            const int64_t ak = av;
            const int64_t ek = kk < ND ? (int64_t)dv : F - 1;
            const double ts = sw_mid(f.st, f.step, f.dur, ak), te = sw_mid(f.st, f.step, f.dur, ek);
            s = ts - a.pad_on;
            e = te + a.pad_off;
            return (te - ts) > a.maxd ? 2 : ((e - s) > 1e-6 ? 1 : 0);
        };
        // a chunk's list loads issued together
        auto chunk = [&](int64_t kc, int32_t* av, int32_t* dv) {
#pragma unroll
            for (int j = 0; j < 2 * kBinChunk; ++j) {
                const int64_t kk = min<int64_t>(kc + j, k1 - 1);
                av[j] = ra[kk];
                dv[j] = rd[min<int64_t>(kk, ND > 0 ? ND - 1 : 0)];
            }
        };
        int64_t cnt_put = 0;
        int any_long = 0;
        for (int64_t kc = k0; kc < k1; kc += 2 * kBinChunk) {
            int32_t av[2 * kBinChunk], dv[2 * kBinChunk];
            chunk(kc, av, dv);
#pragma unroll
            for (int j = 0; j < 2 * kBinChunk; ++j) {
                if (kc + j >= k1) break;
                double s, e;
                const int c = region(kc + j, av[j], dv[j], s, e);
                any_long |= c == 2;
                cnt_put += c == 1;
            }
        }
        if (!__syncthreads_or(any_long)) {
            unsigned long long tot;
            const unsigned long long p0 = wg_exclusive_scan(
                (unsigned long long)cnt_put, 0ull, [](unsigned long long x, unsigned long long y) { return x + y; },
                s_n, tot);
            int64_t p = (int64_t)p0;
            for (int64_t kc = k0; kc < k1; kc += 2 * kBinChunk) {
                int32_t av[2 * kBinChunk], dv[2 * kBinChunk];
                chunk(kc, av, dv);
#pragma unroll
                for (int j = 0; j < 2 * kBinChunk; ++j) {
                    if (kc + j >= k1) break;
                    double s, e;
                    if (region(kc + j, av[j], dv[j], s, e) == 1) {
                        if (p < cap) {
                            rs[p] = s;
                            re[p] = e;
                        }
                        ++p;
                    }
                }
            }
            if (t == 0) a.reg_count[file] = (int64_t)tot > cap ? -1 : (int64_t)tot;
            return;
        }
    }
    if (t >= kWave) return;

    // ---- wave 0: regions in order, 64 per batch
    f.zw = Z;
    f.nw = nb;
    f.mv = sa.w.mv + wb;
    f.mi = sa.w.mi + wb;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int64_t pos = 0, k = 0, last_deact = 0;  // frame 0 is the stale score before a first activation
    bool overflow = false;
    int64_t flushed = 0;  // regions [0, flushed) are out of the ring
    auto flush_to = [&](int64_t upto) {
        for (int64_t q = flushed + lane; q < upto && q < cap; q += kWave) {
            rs[q] = s_rs[q & (kBinRing - 1)];
            re[q] = s_re[q & (kBinRing - 1)];
        }
        flushed = upto;
    };
    // the next batch's lists are loaded one batch ahead (clamped, unconditional loads)
    auto ld_a = [&](int64_t j) { return ra[min<int64_t>(j, R - 1)]; };
    auto ld_d = [&](int64_t j) { return rd[min<int64_t>(j, ND > 0 ? ND - 1 : 0)]; };
    int64_t pk = k;
    int32_t pa = R > 0 ? ld_a(k + lane) : 0, pd = R > 0 ? ld_d(k + lane) : 0;
    while (k < R) {
        k = uniform64(k);
        const int64_t kk = k + lane;
        const bool valid = kk < R;
        int32_t ca = pa, cd = pd;
        if (pk != k) {
            ca = ld_a(kk);
            cd = ld_d(kk);
        }
        pk = k + kWave;
        pa = ld_a(pk + lane);
        pd = ld_d(pk + lane);
        const int64_t ak = valid ? (int64_t)ca : 0;
        const int64_t dk = (valid && kk < ND) ? (int64_t)cd : -1;
        const int64_t ek = dk >= 0 ? dk : F - 1;
        const double ts = sw_mid(f.st, f.step, f.dur, ak), te = sw_mid(f.st, f.step, f.dur, ek);
        const unsigned long long lm = __ballot(valid && (te - ts) > a.maxd);
        const int nn = lm ? __ffsll((long long)lm) - 1 : kWave;  // regions before the first long one
        const double s = ts - a.pad_on, e = te + a.pad_off;
        const bool put = valid && lane < nn && (e - s) > 1e-6;
        const unsigned long long pm = __ballot(put);
        if (pos + kWave - flushed > kBinRing) flush_to(pos);
        const int64_t p = pos + __popcll(pm & lt);
        if (put) {
            s_rs[p & (kBinRing - 1)] = s;
            s_re[p & (kBinRing - 1)] = e;
        }
        pos += __popcll(pm);
        const int m = (int)min<int64_t>(nn, R - k);
        if (m > 0) last_deact = uniform64(__shfl(dk, m - 1));
        k += m;
        if (!lm || k >= R) continue;
        // region k exceeds max_duration: the sequential machine from its activation
        const int64_t a0 = uniform64(__shfl(ak, nn));
        flush_to(pos);
        const int64_t room = pos < cap ? cap - pos : 0;
        RegionOut out{rs + (cap - room), re + (cap - room), room};
        const int64_t dstar = bin_active_run(a, f, sw_mid(f.st, f.step, f.dur, a0), a0 != 0, last_deact,
                                             a0 == 0 ? 0 : a0 + 1, a0 + 1, out, lane);
        out.flush(lane);
        overflow |= out.overflow;
        pos += out.n;
        flushed = pos;
        if (dstar < 0) break;
        last_deact = dstar;
        // resume at the first region activated after dstar
        int64_t j0 = k + 1;
        while (true) {
            j0 = uniform64(j0);
            const int64_t jj = j0 + lane;
            const bool after = jj < R && (int64_t)ra[jj] > dstar;
            const unsigned long long am = __ballot(after);
            if (am) {
                k = j0 + __ffsll((long long)am) - 1;
                break;
            }
            j0 += kWave;
            if (j0 >= R) {
                k = R;
                break;
            }
        }
    }
    flush_to(pos);
    if (lane == 0) a.reg_count[file] = (overflow || pos > cap) ? -1 : pos;
}

}  // namespace wx

namespace wx {
// Column 0 of get_trellis (alignment.py:367): S(t) = em[0, c] + ... + em[t - 1, c] in double,
// row order, t = 0..T — the fused DP's own column-0 routine (col0_chunk: binade scan, else the
// sequential chain), one wave.  Rows past T in the last chunk enter as 0 and feed only sums
// past S(T), which are not stored.
__global__ __launch_bounds__(kWave) void column0_cumsum_kernel(const float* __restrict__ em, int64_t T, int V,
                                                               double* __restrict__ S) {
    const int l = lane_id();
    double acc = 0.0;
    for (int64_t t0 = 0; t0 < T; t0 += kChunk) {
        const int64_t t = t0 + (l & (kChunk - 1));
        const float e = t < T ? em[t * V] : 0.0f;
        const double a = col0_chunk(acc, e);
        if (l < kChunk) S[t0 + l] = a;  // S(t0 + l), t0 + l < T
    }
    if (l == 0) S[T] = acc;
}
}  // namespace wx

// ======================================================================================
// C ABI
namespace wx {
// ------------------------------------------------------------------------------------
// VAD producer: overlap-add aggregation of the segmentation model's per-chunk frame scores
// onto the file's frame grid (pyannote.audio Inference.aggregate, as called by
// VoiceActivityDetection / whisperx's VoiceActivitySegmentation.apply, vad.py:198-240), with
// the multi-label pre-aggregation hook (max over the model's speaker classes) fused in.
// One thread per output frame gathers the chunks covering it in chunk order (the
// reference's accumulation order: chunk by chunk, fp32 `+=`), so the result is deterministic
// and equals the sequential numpy sum bit for bit.  Chunk c covers output frames
// [start_frame[c], start_frame[c] + K); start_frame is non-decreasing.
struct VadAggArgs {
    const float* scores;        // [n_chunks, K, n_classes]
    const int64_t* start_frame; // [n_chunks]
    int n_chunks, K, n_classes;
    int64_t n_frames;
    float missing;              // value of frames no chunk covers (or all-NaN)
    float* out;                 // [n_frames]
};

__global__ __launch_bounds__(256) void vad_aggregate_kernel(VadAggArgs a) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= a.n_frames) return;
    // first chunk whose window can reach frame f: start_frame[c] > f - K (binary search)
    int lo = 0, hi = a.n_chunks;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a.start_frame[mid] <= f - a.K) lo = mid + 1;
        else hi = mid;
    }
    float acc = 0.0f, cnt = 0.0f;
    bool any = false;
    for (int c = lo; c < a.n_chunks; ++c) {
        const int64_t s0 = a.start_frame[c];
        if (s0 > f) break;
        const int i = (int)(f - s0);
        if (i >= a.K) continue;
        const float* row = a.scores + ((int64_t)c * a.K + i) * a.n_classes;
        float m = row[0];
        for (int k = 1; k < a.n_classes; ++k) {
            const float v = row[k];
            m = (m != m || v != v) ? __builtin_nanf("") : fmaxf(m, v);  // np.max: NaN propagates
        }
        if (m == m) {  // mask = 1 - isnan
            acc = acc + m;
            cnt = cnt + 1.0f;
            any = true;
        }
    }
    a.out[f] = any ? acc / fmaxf(cnt, 1e-12f) : a.missing;
}
}  // namespace wx

using namespace wx;

namespace {

int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }


// Kernels of different (C, W) buckets are independent: a batch that spans several buckets
// forks them onto a small per-device pool of non-blocking streams and joins back onto the
// caller's stream with events, so they run concurrently (a latency-bound batch then costs
// the slowest bucket, not their sum).  Created once per device; enqueue is serialised by
// a mutex so concurrent callers cannot interleave fork/join events.
struct ForkPool {
    static constexpr int kMax = 12;
    hipStream_t s[kMax];
    hipEvent_t fork;
    hipEvent_t join[kMax];
    std::mutex mu;
};

ForkPool* fork_pool() {
    static std::mutex mu;
    static ForkPool* pools[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!pools[dev]) {
        ForkPool* p = new ForkPool;
        bool ok = hipEventCreateWithFlags(&p->fork, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < ForkPool::kMax; ++i) {
            ok = hipStreamCreateWithFlags(&p->s[i], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&p->join[i], hipEventDisableTiming) == hipSuccess;
        }
        if (!ok) return nullptr;
        pools[dev] = p;
    }
    return pools[dev];
}

// Run launch(i, stream) for i in [0, n): on the caller's stream when n == 1, otherwise
// forked over the pool and joined back onto `st`.
template <class F>
int fork_join(hipStream_t st, int n, F&& launch) {
    if (n <= 0) return WX_OK;
    if (n == 1) {
        launch(0, st);
        return launch_status();
    }
    ForkPool* p = fork_pool();
    if (!p || n > ForkPool::kMax) {  // serial fallback on the caller's stream
        for (int i = 0; i < n; ++i) launch(i, st);
        return launch_status();
    }
    std::lock_guard<std::mutex> g(p->mu);
    hipError_t e = hipEventRecord(p->fork, st);
    for (int i = 0; i < n && e == hipSuccess; ++i) {
        e = hipStreamWaitEvent(p->s[i], p->fork, 0);
        if (e != hipSuccess) break;
        launch(i, p->s[i]);
        e = hipEventRecord(p->join[i], p->s[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, p->join[i], 0);
    }
    const int rc = launch_status();
    return e != hipSuccess ? (int)e : rc;
}

// bucket ids in launch order, ids = C*64 + W
constexpr int kBucketIds[] = {
#define WX_ID(CC, WW, HH) bucket_make(CC, WW, HH),
    WX_BUCKETS(WX_ID)
#undef WX_ID
};
constexpr int kNumBuckets = sizeof(kBucketIds) / sizeof(int);

// The buckets that segments with N in [min_N, max_N] map to (N == 0 -> the first one).
int buckets_for(int64_t min_N, int64_t max_N, int mode, int* ids) {
    int n = 0;
    int64_t N = std::max<int64_t>(min_N, 1);
    const int64_t hi = std::max<int64_t>(max_N, 1);
    while (N <= hi) {
        const int id = bucket_id((int)N, mode);
        ids[n++] = id;
        N = (int64_t)bucket_capacity(bucket_C(id), bucket_W(id)) + 1;
    }
    return n;
}

// The split launch's one split bucket, for a batch whose longest segment has max_N tokens.
int split_launch_id(int64_t max_N, int P) {
    const int id = split_bucket_id((int)std::min<int64_t>(std::max<int64_t>(max_N, 1), 1 << 20), P);
    if (id & kSplitFlag) return id;
    int widest = 0;
#define WX_WIDEST(CC, WW) widest = bucket_make(CC, WW, 1) | kSplitFlag;
    WX_SPLIT_BUCKETS(WX_WIDEST)
#undef WX_WIDEST
    return widest;
}

// Kernels of a split launch: the split bucket, then the single-CU latency buckets of any
// segment too long for it.
int buckets_for_split(int64_t min_N, int64_t max_N, int P, int split_id, int* ids) {
    int n = 0;
    ids[n++] = split_id;
    const int64_t cap = split_capacity_of(split_id, P);
    const int C = bucket_C(split_id & ~kSplitFlag);
    const int64_t small_hi = std::min<int64_t>(max_N, (int64_t)C * (C - 1));  // layout_fits holds above
    if (C > 2 && min_N <= small_hi) n += buckets_for(min_N, small_hi, WX_MODE_THROUGHPUT, ids + n);
    if (max_N > cap) n += buckets_for(std::max<int64_t>(min_N, cap + 1), max_N, WX_MODE_LATENCY, ids + n);
    return n;
}

// bitmap words per block of the bucket `id` of an N-token segment in a launch of P parts
int launch_cells_total(int id, int P) {
    return (id & kSplitFlag) ? bucket_cells_total(id & ~kSplitFlag) * P : bucket_cells_total(id);
}

// bitmap: per segment (floor(row0/32) + seg) block offsets, 64 * C_stride dwords per block
size_t bitmap_bytes(int32_t S, int64_t sum_T, int64_t max_N, int* stride_cells) {
    const int nmax = (int)std::max<int64_t>(max_N, 1);  // widest bucket of any launch shape
    int cells = std::max(bucket_cells_total(bucket_id(nmax, 0)), bucket_cells_total(bucket_id(nmax, 1)));
    for (int P = 2; P <= kMaxParts; ++P) cells = std::max(cells, launch_cells_total(split_launch_id(nmax, P), P));
    if (stride_cells) *stride_cells = cells;
    const int64_t blocks = sum_T / kChunk + S + 1;
    return align_up((size_t)blocks * (size_t)cells * 4u, 256);
}

}  // namespace

extern "C" {

const char* wx_version(void) { return WX_VERSION " gfx950"; }

const char* wx_strerror(int code) {
    switch (code) {
        case WX_OK: return "ok";
        case WX_E_INVALID: return "invalid argument";
        case WX_E_VOCAB: return "vocabulary size outside [1, 16384]";
        case WX_E_TOO_LONG: return "segment has more than 16000 tokens";
        case WX_E_WORKSPACE: return "workspace too small";
        case WX_E_LAUNCH: return "kernel launch failed";
        default: return hipGetErrorString((hipError_t)code);
    }
}

// Launch shape: latency buckets while the batch cannot fill the chip with one wave per
// segment.  WX_ALIGN_MODE=0/1 forces a shape for WX_MODE_AUTO calls (benchmarking only).
int align_mode(int32_t S, int32_t mode) {
    if (mode == WX_MODE_THROUGHPUT) return mode;
    if (mode != WX_MODE_AUTO) return WX_MODE_LATENCY;  // LATENCY, LATENCY_1CU, SPLIT2..4
    static const int forced = [] {
        const char* e = getenv("WX_ALIGN_MODE");
        return (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : -1;
    }();
    if (forced >= 0) return forced;
    return S <= 256 ? WX_MODE_LATENCY : WX_MODE_THROUGHPUT;
}

size_t cmask_bytes(int32_t S, int64_t sum_T) { return align_up((size_t)(sum_T / kChunk + S + 1) * 4u, 256); }

// column N history: segment s at (row0 + 4 s) & ~3 (16-byte aligned groups of 8 rows)
size_t cn_bytes(int32_t S, int64_t sum_T) { return align_up((size_t)(sum_T + kCnPad * (int64_t)S + 16) * 4u, 256); }

// split hand-off granules: per (floor(row0/32) + seg + chunk) block, 3 boundaries x 40
size_t xg_bytes(int32_t S, int64_t sum_T) {
    return align_up((size_t)(sum_T / kChunk + S + 2) * (kMaxParts - 1) * kHaloCells * 8u, 256);
}
size_t arrive_bytes(int32_t S) { return align_up((size_t)(S + 1) * 8u, 256); }
// checkpointed kernels' column-0 cumsum per chunk: (floor(row0/32) + seg + q) doubles
size_t c0acc_bytes(int32_t S, int64_t sum_T) { return align_up((size_t)(sum_T / kChunk + S + 2) * 8u, 256); }

size_t wx_align_dp_workspace_bytes(int32_t S, int64_t sum_T, int64_t max_N) {
    return bitmap_bytes(S, sum_T, max_N, nullptr) + align_up((size_t)(sum_T + 1) * 4u, 256) + cmask_bytes(S, sum_T) +
           cn_bytes(S, sum_T) + c0acc_bytes(S, sum_T) + xg_bytes(S, sum_T) + arrive_bytes(S);
}

// CUs of the current device (cached per device).
int device_cus() {
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

// Parts per segment of a latency launch.  WX_MODE_AUTO splits each segment over 4 CUs when
// the device has 4 CUs per segment (S <= 64 on MI355X), else one CU; WX_MODE_LATENCY is one CU
// unless WX_PARTS=2..4 asks for a split; WX_MODE_SPLIT2..4 ask explicitly.  Measured (T=1499
// and T=2999 segments, round 1): 4 parts take 90 / 101 / 210 us for 16 x 1499 / 64 x 1499 /
// 64 x 2999 against 107 / 110 / 309 us on one CU; 2 or 3 parts gain nothing (they pick C=2
// buckets, whose step is as long as the one-CU bucket's).  Every part stages all emission
// rows (4x the emission reads, ~0.5 TB/s at config 2: far from any bound).  The CU count
// caps the parts: part p only waits for part p-1, which the dispatcher starts first.
int split_parts(int32_t S, int mode, int32_t requested) {
    static const int forced = [] {
        const char* e = getenv("WX_PARTS");
        return (e && e[0] >= '1' && e[0] <= '0' + kMaxParts) ? e[0] - '0' : 0;
    }();
    if (mode != WX_MODE_LATENCY) return 1;
    if (requested == WX_MODE_LATENCY_1CU) return 1;
    const int fit = device_cus() / std::max(S, 1);
    int want = 1;
    if (requested >= WX_MODE_SPLIT2 && requested <= WX_MODE_SPLIT4)
        want = requested - WX_MODE_SPLIT2 + 2;
    else if (forced)
        want = forced;
    else if (requested == WX_MODE_AUTO && fit >= kMaxParts)
        want = kMaxParts;
    if (want <= 1) return 1;
    return std::max(1, std::min(want, fit)) >= 2 ? std::max(1, std::min(want, fit)) : 1;
}

unsigned next_epoch() {  // never 0: a zeroed granule or counter carries no valid tag
    static std::atomic<unsigned> e{(unsigned)std::chrono::steady_clock::now().time_since_epoch().count()};
    const unsigned v = e.fetch_add(1) + 1;
    return v ? v : 1u;
}

// Hand-off re-reads before a split part gives up on a granule.  WX_SPIN_LIMIT (read per call)
// lowers it; 0 forces every consumer to lose its hand-offs (the recovery test).
static int spin_limit() {
    const char* e = getenv("WX_SPIN_LIMIT");
    if (e && e[0] >= '0' && e[0] <= '9') return std::min(atoi(e), kMaxSpin);
    return kMaxSpin;
}
// Split-arrival flags, read per call (tests and A/B): WX_SPLIT_FENCED=1 adds the release /
// acquire fences to the write-through arrival, WX_SPLIT_XCD_SPREAD=1 spreads each segment's
// parts over different XCDs.
static int split_flags() {
    auto on = [](const char* n) {
        const char* e = getenv(n);
        return e && e[0] == '1';
    };
    return (on("WX_SPLIT_FENCED") ? kArgFenced : 0) | (on("WX_SPLIT_XCD_SPREAD") ? kArgXcdSpread : 0);
}

size_t wx_align_dp_handoff_bytes(int32_t S, int64_t sum_T) { return xg_bytes(S, sum_T) + arrive_bytes(S); }

int wx_align_dp(const float* em, const int64_t* em_off, int32_t V, const int32_t* tok, const int64_t* tok_off,
                const int32_t* blank_id, int32_t S, int64_t min_N, int64_t max_N, int64_t sum_T, int32_t* seg_start,
                int32_t* seg_end, double* seg_score, int32_t* t_start, int32_t* status, void* workspace,
                size_t workspace_bytes, void* stream) {
    return wx_align_dp_mode(em, em_off, V, tok, tok_off, blank_id, S, min_N, max_N, sum_T, seg_start, seg_end,
                            seg_score, t_start, status, workspace, workspace_bytes, WX_MODE_AUTO, stream);
}

int wx_align_dp_mode(const float* em, const int64_t* em_off, int32_t V, const int32_t* tok,
                     const int64_t* tok_off, const int32_t* blank_id, int32_t S, int64_t min_N, int64_t max_N,
                     int64_t sum_T, int32_t* seg_start, int32_t* seg_end, double* seg_score, int32_t* t_start,
                     int32_t* status, void* workspace, size_t workspace_bytes, int32_t mode, void* stream) {
    return wx_align_dp_ex(em, em_off, V, tok, tok_off, blank_id, S, min_N, max_N, sum_T, seg_start, seg_end,
                          seg_score, t_start, status, workspace, workspace_bytes, nullptr, 0, mode, stream);
}

int wx_align_dp_ex(const float* em, const int64_t* em_off, int32_t V, const int32_t* tok,
                   const int64_t* tok_off, const int32_t* blank_id, int32_t S, int64_t min_N, int64_t max_N,
                   int64_t sum_T, int32_t* seg_start, int32_t* seg_end, double* seg_score, int32_t* t_start,
                   int32_t* status, void* workspace, size_t workspace_bytes, void* handoff, size_t handoff_bytes,
                   int32_t mode, void* stream) {
    if (!(mode >= WX_MODE_AUTO && mode <= WX_MODE_LATENCY_1CU) && !(mode >= WX_MODE_SPLIT2 && mode <= WX_MODE_SPLIT4))
        return WX_E_INVALID;
    if (S < 0 || sum_T < 0 || min_N < 0 || max_N < min_N) return WX_E_INVALID;
    if (S == 0) return WX_OK;
    if (!em || !em_off || !tok_off || !blank_id || !seg_start || !seg_end || !seg_score || !t_start || !status ||
        !workspace)
        return WX_E_INVALID;
    if (V < 1 || V > WX_MAX_VOCAB) return WX_E_VOCAB;
#ifdef WX_DEV_V32
    if (V > 32) return WX_E_INVALID;  // development build: only the V <= 32 kernels exist
#endif
    if (max_N > WX_MAX_TOKENS) return WX_E_TOO_LONG;
    if (workspace_bytes < wx_align_dp_workspace_bytes(S, sum_T, max_N)) return WX_E_WORKSPACE;
    if (handoff && handoff_bytes < wx_align_dp_handoff_bytes(S, sum_T)) return WX_E_WORKSPACE;
    AlignArgs a;
    a.em = em; a.em_off = em_off; a.V = V; a.tok = tok; a.tok_off = tok_off; a.blank_id = blank_id; a.S = S;
    a.seg_start = seg_start; a.seg_end = seg_end; a.seg_score = seg_score; a.t_start = t_start; a.status = status;
    const size_t bm = bitmap_bytes(S, sum_T, max_N, &a.bits_stride_cells);
    a.bits = reinterpret_cast<unsigned*>(workspace);
    a.q0 = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + bm);
    a.cmask = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(workspace) + bm +
                                          align_up((size_t)(sum_T + 1) * 4u, 256));
    a.cn = reinterpret_cast<float*>(reinterpret_cast<char*>(a.cmask) + cmask_bytes(S, sum_T));
    a.c0acc = reinterpret_cast<double*>(reinterpret_cast<char*>(a.cn) + cn_bytes(S, sum_T));
    a.xg = reinterpret_cast<uint64_t*>(handoff ? handoff : reinterpret_cast<char*>(a.c0acc) + c0acc_bytes(S, sum_T));
    a.arrive = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.xg) + xg_bytes(S, sum_T));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    a.mode = align_mode(S, mode);
    a.parts = split_parts(S, a.mode, mode);
    a.epoch = next_epoch();
    a.spin = spin_limit();
    a.flags = split_flags();
    if (a.parts > 1 && !handoff) {  // workspace hand-off region: holds anything until zeroed
        const hipError_t e = hipMemsetAsync(a.xg, 0, wx_align_dp_handoff_bytes(S, sum_T), st);
        if (e != hipSuccess) return (int)e;
    }
    a.x4 = (V == 32 && (reinterpret_cast<uintptr_t>(em) & 15) == 0) ? 1 : 0;
    int ids[kNumBuckets + 8];
    a.split_id = a.parts > 1 ? split_launch_id(max_N, a.parts) : 0;
    const int n = a.parts > 1 ? buckets_for_split(min_N, max_N, a.parts, a.split_id, ids)
                              : buckets_for(min_N, max_N, a.mode, ids);
    const dim3 grid(S);
    return fork_join(st, n, [&](int i, hipStream_t s) {
#define WX_LAUNCH_SPLIT(CC, WW)                                                                        \
        if (ids[i] == (bucket_make(CC, WW, 1) | kSplitFlag)) {                                          \
            const dim3 g2(split_grid(S, a.parts));                                                        \
            if (V <= 32) launch_align_split<CC, 32, WW>(g2, s, a);                                         \
            else if (V <= 64) launch_align_split<CC, WX_VS64, WW>(g2, s, a);                                \
            else launch_align_split<CC, WX_VSG, WW>(g2, s, a);                                            \
        }
        WX_SPLIT_BUCKETS(WX_LAUNCH_SPLIT)
#undef WX_LAUNCH_SPLIT
#define WX_LAUNCH_ALIGN(CC, WW, HH)                                                                  \
        if (ids[i] == bucket_make(CC, WW, HH)) {                                                       \
            if (V <= 32) launch_align_dp<CC, 32, WW, HH>(grid, s, a);                                  \
            else if (V <= 64) launch_align_dp<CC, WX_VS64, WW, HH>(grid, s, a);                             \
            else launch_align_dp<CC, WX_VSG, WW, HH>(grid, s, a);                                   \
        }
        WX_BUCKETS(WX_LAUNCH_ALIGN)
#undef WX_LAUNCH_ALIGN
    });
}

int wx_align_dp_plan(int32_t S, int64_t min_N, int64_t max_N, int32_t V, int32_t mode, char* buf, size_t n) {
    if (S <= 0 || min_N < 0 || max_N < min_N || V < 1) return 0;
    const int m = align_mode(S, mode);
    const int P = split_parts(S, m, mode);
    int ids[kNumBuckets + 8];
    const int cnt = P > 1 ? buckets_for_split(min_N, max_N, P, split_launch_id(max_N, P), ids)
                          : buckets_for(min_N, max_N, m, ids);
    const int vs = V <= 32 ? 32 : (V <= 64 ? 64 : kGatherVS);
    size_t used = 0;
    for (int i = 0; i < cnt && buf && n > 0; ++i) {
        const int id = ids[i] & ~kSplitFlag;
        char one[160];
        if (ids[i] & kSplitFlag)
            snprintf(one, sizeof one, "%svoid wx::align_dp_split_kernel<%d, %d, %d>(wx::AlignArgs)", i ? ";" : "",
                     bucket_C(id), vs, bucket_W(id));
        else
            snprintf(one, sizeof one, "%svoid wx::align_dp_kernel<%d, %d, %d, %d>(wx::AlignArgs)", i ? ";" : "",
                     bucket_C(id), vs, bucket_W(id), id & 1);
        const size_t len = strlen(one);
        if (used + len + 1 > n) break;
        memcpy(buf + used, one, len + 1);
        used += len;
    }
    return cnt;
}

int wx_trellis(const float* em, const int64_t* em_off, int32_t V, const int32_t* tok, const int64_t* tok_off,
               const int32_t* blank_id, int32_t S, int64_t max_N, float* trellis, const int64_t* tr_off,
               void* stream) {
    if (S < 0 || max_N < 0) return WX_E_INVALID;
    if (S == 0) return WX_OK;
    if (!em || !em_off || !tok_off || !blank_id || !trellis || !tr_off) return WX_E_INVALID;
    if (V < 1 || V > WX_MAX_VOCAB) return WX_E_VOCAB;
#ifdef WX_DEV_V32
    if (V > 32) return WX_E_INVALID;  // development build: only the V <= 32 kernels exist
#endif
    if (max_N > WX_MAX_TOKENS) return WX_E_TOO_LONG;
    TrellisArgs a;
    a.em = em; a.em_off = em_off; a.V = V; a.tok = tok; a.tok_off = tok_off; a.blank_id = blank_id;
    a.tr = trellis; a.tr_off = tr_off;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    a.x4 = (V == 32 && (reinterpret_cast<uintptr_t>(em) & 15) == 0) ? 1 : 0;
    int ids[kNumBuckets];
    const int n = buckets_for(0, max_N, 0, ids);
    const dim3 grid(S);
    return fork_join(st, n, [&](int i, hipStream_t s) {
#define WX_LAUNCH_TR(CC, WW, HH)                                                                        \
        if (!HH && ids[i] == bucket_make(CC, WW, 0)) {                                                \
            if (V <= 32) launch_trellis<CC, 32, WW>(grid, s, a);                                         \
            else if (V <= 64) launch_trellis<CC, WX_VS64, WW>(grid, s, a);                               \
            else launch_trellis<CC, WX_VSG, WW>(grid, s, a);                                            \
        }
        WX_BUCKETS(WX_LAUNCH_TR)
#undef WX_LAUNCH_TR
    });
}

size_t wx_backtrack_workspace_bytes(int32_t S, int64_t sum_T, int64_t max_N) {
    const int64_t cpl = std::max<int64_t>(1, (max_N + kWave - 1) / kWave);
    const int64_t blocks = sum_T / kChunk + S + 1;
    // bitmap + per-token start frames (sum of N <= S * max_N)
    return align_up((size_t)blocks * kWave * (size_t)cpl * 4u, 256) + align_up((size_t)(S * max_N + 1) * 4u, 256) +
           cmask_bytes(S, sum_T);
}

int wx_backtrack(const float* trellis, const int64_t* tr_off, const float* em, const int64_t* em_off, int32_t V,
                 const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id, int32_t S, int64_t max_N,
                 int64_t sum_T, int32_t* path_tok, int32_t* path_time, float* path_prob, int32_t* path_len,
                 int32_t* t_start, void* workspace, size_t workspace_bytes, void* stream) {
    if (S < 0 || max_N < 0 || sum_T < 0) return WX_E_INVALID;
    if (S == 0) return WX_OK;
    if (!trellis || !tr_off || !em || !em_off || !tok_off || !blank_id || !path_tok || !path_time || !path_prob ||
        !path_len || !t_start || !workspace)
        return WX_E_INVALID;
    if (V < 1) return WX_E_VOCAB;
    if (workspace_bytes < wx_backtrack_workspace_bytes(S, sum_T, max_N)) return WX_E_WORKSPACE;
    BacktrackArgs a;
    a.tr = trellis; a.tr_off = tr_off; a.em = em; a.em_off = em_off; a.V = V; a.tok = tok; a.tok_off = tok_off;
    a.blank_id = blank_id; a.path_tok = path_tok; a.path_time = path_time; a.path_prob = path_prob;
    a.path_len = path_len; a.t_start = t_start;
    const int64_t cpl = std::max<int64_t>(1, (max_N + kWave - 1) / kWave);
    a.bits_stride_cells = (int)(kWave * cpl);
    const int64_t blocks = sum_T / kChunk + S + 1;
    const size_t bm = align_up((size_t)blocks * kWave * (size_t)cpl * 4u, 256);
    a.bits = reinterpret_cast<unsigned*>(workspace);
    a.start = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(workspace) + bm);
    a.cmask = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(workspace) + bm +
                                          align_up((size_t)(S * max_N + 1) * 4u, 256));
    hipLaunchKernelGGL(backtrack_kernel, dim3(S), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launch_status();
}

int wx_merge_repeats(const int32_t* path_tok, const int32_t* path_time, const float* path_prob,
                     const int64_t* path_off, const int32_t* path_len, int32_t S, int32_t* seg_tok,
                     int32_t* seg_start, int32_t* seg_end, double* seg_score, int32_t* seg_count, void* stream) {
    if (S < 0) return WX_E_INVALID;
    if (S == 0) return WX_OK;
    if (!path_tok || !path_time || !path_prob || !path_off || !path_len || !seg_tok || !seg_start || !seg_end ||
        !seg_score || !seg_count)
        return WX_E_INVALID;
    MergeArgs a;
    a.ptok = path_tok; a.ptime = path_time; a.pprob = path_prob; a.path_off = path_off; a.path_len = path_len;
    a.seg_tok = seg_tok; a.seg_start = seg_start; a.seg_end = seg_end; a.seg_score = seg_score;
    a.seg_count = seg_count;
    hipLaunchKernelGGL(merge_repeats_kernel, dim3(S), dim3(kWave), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launch_status();
}

int wx_column0_cumsum(const float* em, int64_t T, int32_t V, double* S, void* stream) {
    if (T < 0 || V < 1 || !S || (T > 0 && !em)) return WX_E_INVALID;
    hipLaunchKernelGGL(column0_cumsum_kernel, dim3(1), dim3(kWave), 0, reinterpret_cast<hipStream_t>(stream), em, T,
                       V, S);
    return launch_status();
}

int wx_binarize(const float* scores, const int64_t* f_off, int32_t n_files, const double* sw_start,
                const double* sw_step, const double* sw_duration, float onset, float offset, double max_duration,
                double pad_onset, double pad_offset, double* reg_start, double* reg_end, const int64_t* reg_off,
                int64_t* reg_count, void* stream) {
    if (n_files < 0) return WX_E_INVALID;
    if (n_files == 0) return WX_OK;
    if (!scores || !f_off || !sw_start || !sw_step || !sw_duration || !reg_start || !reg_end || !reg_off ||
        !reg_count)
        return WX_E_INVALID;
    BinarizeArgs a;
    a.y = scores; a.f_off = f_off; a.sw_start = sw_start; a.sw_step = sw_step; a.sw_dur = sw_duration;
    a.onset = onset; a.offset = offset; a.maxd = max_duration; a.pad_on = pad_onset; a.pad_off = pad_offset;
    a.rs = reg_start; a.re = reg_end; a.reg_off = reg_off; a.reg_count = reg_count;
    hipLaunchKernelGGL(binarize_kernel, dim3(n_files), dim3(kWave), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launch_status();
}

// offset <= onset: no frame both sets and resets the state, so the parallel scan is exact
static bool binarize_uses_scan(float onset, float offset) { return offset <= onset; }

size_t wx_binarize_workspace_bytes(int32_t n_files, int64_t total_frames) {
    if (n_files < 0 || total_frames < 0) return 0;
    const size_t nw = (size_t)bin_words(total_frames, n_files);
    const size_t nl = (size_t)total_frames + (size_t)n_files;  // region lists, F + 1 per file
    return 2 * align_up(nw * 8u, 256) + 2 * align_up(nw * 4u, 256) + 2 * align_up(nl * 4u, 256);
}

int wx_binarize_ex(const float* scores, const int64_t* f_off, int32_t n_files, int64_t total_frames,
                   const double* sw_start, const double* sw_step, const double* sw_duration, float onset, float offset,
                   double max_duration, double pad_onset, double pad_offset, double* reg_start, double* reg_end,
                   const int64_t* reg_off, int64_t* reg_count, void* workspace, size_t workspace_bytes,
                   void* stream) {
    if (n_files < 0 || total_frames < 0) return WX_E_INVALID;
    if (n_files == 0) return WX_OK;
    if (!scores || !f_off || !sw_start || !sw_step || !sw_duration || !reg_start || !reg_end || !reg_off ||
        !reg_count || !workspace)
        return WX_E_INVALID;
    if (workspace_bytes < wx_binarize_workspace_bytes(n_files, total_frames)) return WX_E_WORKSPACE;
    const int64_t nw = bin_words(total_frames, n_files);
    char* p = reinterpret_cast<char*>(workspace);
    BinWords w;
    w.on = reinterpret_cast<unsigned long long*>(p);
    p += align_up((size_t)nw * 8u, 256);
    w.off = reinterpret_cast<unsigned long long*>(p);
    p += align_up((size_t)nw * 8u, 256);
    w.mv = reinterpret_cast<float*>(p);
    p += align_up((size_t)nw * 4u, 256);
    w.mi = reinterpret_cast<int32_t*>(p);
    p += align_up((size_t)nw * 4u, 256);
    const size_t nl = (size_t)total_frames + (size_t)n_files;
    int32_t* ra = reinterpret_cast<int32_t*>(p);
    p += align_up(nl * 4u, 256);
    int32_t* rd = reinterpret_cast<int32_t*>(p);
    BinWordArgs wa;
    wa.y = scores; wa.f_off = f_off; wa.n_files = n_files; wa.n_words = nw; wa.onset = onset; wa.offset = offset;
    wa.w = w;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (total_frames > 0)  // (its tile loads read frame 0 for words past a file's end)
        hipLaunchKernelGGL(binarize_words_kernel, dim3((unsigned)((nw + kWave - 1) / kWave)), dim3(kWave), 0, s, wa);
    BinarizeArgs a;
    a.y = scores; a.f_off = f_off; a.sw_start = sw_start; a.sw_step = sw_step; a.sw_dur = sw_duration;
    a.onset = onset; a.offset = offset; a.maxd = max_duration; a.pad_on = pad_onset; a.pad_off = pad_offset;
    a.rs = reg_start; a.re = reg_end; a.reg_off = reg_off; a.reg_count = reg_count;
    if (binarize_uses_scan(onset, offset)) {
        BinScanArgs sa;
        sa.a = a; sa.w = w; sa.ra = ra; sa.rd = rd;
        hipLaunchKernelGGL(binarize_scan_kernel, dim3(n_files), dim3(kBinWG), 0, s, sa);
    } else {
        hipLaunchKernelGGL(binarize_fsm_kernel, dim3(n_files), dim3(kWave), 0, s, a, w);
    }
    return launch_status();
}

int wx_binarize_plan(float onset, float offset, int64_t total_frames, char* buf, size_t n) {
    const char* words = "void wx::binarize_words_kernel(wx::BinWordArgs)";
    const char* second = binarize_uses_scan(onset, offset) ? "void wx::binarize_scan_kernel(wx::BinScanArgs)"
                                                           : "void wx::binarize_fsm_kernel(wx::BinarizeArgs, wx::BinWords)";
    char all[256];
    const int cnt = total_frames > 0 ? 2 : 1;
    if (total_frames > 0)
        snprintf(all, sizeof all, "%s;%s", words, second);
    else
        snprintf(all, sizeof all, "%s", second);
    if (buf && n > 0) {
        strncpy(buf, all, n - 1);
        buf[n - 1] = 0;
    }
    return cnt;
}

}  // extern "C"

extern "C" int wx_vad_aggregate(const float* scores, const int64_t* start_frame, int32_t n_chunks,
                                int32_t frames_per_chunk, int32_t n_classes, int64_t n_frames, float missing,
                                float* out, void* stream) {
    if (n_chunks < 0 || frames_per_chunk < 1 || n_classes < 1 || n_frames < 0) return WX_E_INVALID;
    if (n_frames == 0) return WX_OK;
    if (!out || (n_chunks > 0 && (!scores || !start_frame))) return WX_E_INVALID;
    VadAggArgs a;
    a.scores = scores; a.start_frame = start_frame; a.n_chunks = n_chunks; a.K = frames_per_chunk;
    a.n_classes = n_classes; a.n_frames = n_frames; a.missing = missing; a.out = out;
    const unsigned blocks = (unsigned)((n_frames + 255) / 256);
    hipLaunchKernelGGL(vad_aggregate_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launch_status();
}

#ifdef WX_PHASE_TIMING
extern "C" int wx_debug_phases(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(wx::wx_phase), sizeof(unsigned long long) * 6 * (size_t)n, 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int wx_debug_cq(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(wx::wx_cq), sizeof(unsigned long long) * 48 * 3 * (size_t)n, 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int wx_debug_loop(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(wx::wx_loop), sizeof(unsigned long long) * wx::kLoopSlots * 3 * (size_t)n, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
