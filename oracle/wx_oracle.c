/*
 * wx_oracle.c — CPU restatement of WhisperX's forced-alignment DP and VAD hysteresis.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker* for the HIP path: it is linked
 * only by tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  The
 * product (whisperx_amd) never loads it; there is no CPU fallback in the product.
 *
 * Pinned against golden vectors produced by the reference itself
 * (tests/golden/make_golden.py, run against /root/reference/whisperx in the build
 * container): tests/test_oracle_golden.py checks every function below bit-for-bit
 * (path probabilities within 1 fp32 ULP: the reference's torch CPU exp is MKL's, this
 * oracle and the GPU use the correctly rounded (float)exp((double)x)).
 *
 * Reference being restated (file:line in /root/reference):
 *   wxo_trellis        whisperx/alignment.py:359-379  get_trellis
 *   wxo_backtrack      whisperx/alignment.py:387-421  backtrack
 *   wxo_merge_repeats  whisperx/alignment.py:438-454  merge_repeats
 *   wxo_align_dp       composition of the three, as align() uses them (alignment.py:242-250)
 *   wxo_binarize       whisperx/vad.py:118-180        Binarize.__call__ (single class,
 *                      max_duration min-cut), timestamps = pyannote SlidingWindow middles
 *
 * Numerics (must match the reference's torch-CPU semantics):
 *   - column 0 = cumsum(emission[:,0]) accumulated in double, rounded per row (torch CPU
 *     cumsum accumulates float in double);
 *   - max = torch.maximum: NaN if either operand is NaN, else the larger;
 *   - backtrack tests `changed > stayed` strictly (ties stay); argmax takes the first
 *     maximum with NaN counted as the maximum;
 *   - compiled with -ffp-contract=off (no FMA anywhere).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline float tmax(float a, float b) {
    if (isnan(a) || isnan(b)) return NAN;
    return (b > a) ? b : a;
}

static inline float prob_exp(float x) { return (float)exp((double)x); }

/* alignment.py:359-379.  tr is [(T+1) x (N+1)] row-major. */
void wxo_trellis(const float* em, int64_t T, int32_t V, const int32_t* tok, int64_t N,
                 int32_t blank, float* tr) {
    const int64_t W = N + 1;
    tr[0] = 0.0f;
    double acc = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        acc += (double)em[t * V + 0];
        tr[(t + 1) * W] = (float)acc;
    }
    /* row 0, columns 1..N (the slice -N: of row 0; N==0 means the whole row) */
    if (N == 0) {
        tr[0] = -INFINITY;
    } else {
        for (int64_t j = 1; j <= N; ++j) tr[j] = -INFINITY;
    }
    /* last N rows of column 0 (the whole column when N==0 or N >= T+1) */
    int64_t first = (N == 0 || N >= T + 1) ? 0 : (T + 1 - N);
    for (int64_t t = first; t <= T; ++t) tr[t * W] = INFINITY;
    for (int64_t t = 0; t < T; ++t) {
        const float eb = em[t * V + blank];
        const float* prev = tr + t * W;
        float* cur = tr + (t + 1) * W;
        for (int64_t j = 1; j <= N; ++j) {
            float stay = prev[j] + eb;
            float chg = prev[j - 1] + em[t * V + tok[j - 1]];
            cur[j] = tmax(stay, chg);
        }
    }
}

/* torch.argmax over a column: first max, NaN counts as the max (first NaN wins). */
static int64_t col_argmax(const float* tr, int64_t T, int64_t W, int64_t j) {
    int64_t best = 0;
    float bv = tr[j];
    if (isnan(bv)) return 0;
    for (int64_t t = 1; t <= T; ++t) {
        float v = tr[t * W + j];
        if (isnan(v)) return t;
        if (v > bv) { bv = v; best = t; }
    }
    return best;
}

/* alignment.py:387-421.  Writes the path in forward (reversed-walk) order.
 * Returns path length, or -1 when the reference returns None.  *t_start_out = argmax. */
int64_t wxo_backtrack(const float* tr, const float* em, int64_t T, int32_t V,
                      const int32_t* tok, int64_t N, int32_t blank,
                      int32_t* ptok, int32_t* ptime, float* pprob, int64_t* t_start_out) {
    const int64_t W = N + 1;
    int64_t j = N;
    int64_t t_start = col_argmax(tr, T, W, j);
    if (t_start_out) *t_start_out = t_start;
    int64_t L = 0;
    int ok = 0;
    /* the walk is recorded backwards in a scratch buffer, then reversed */
    for (int64_t t = t_start; t > 0; --t) {
        float stayed = tr[(t - 1) * W + j] + em[(t - 1) * V + blank];
        float changed = tr[(t - 1) * W + j - 1] + em[(t - 1) * V + tok[j - 1]];
        int c = changed > stayed;
        ptok[L] = (int32_t)(j - 1);
        ptime[L] = (int32_t)(t - 1);
        pprob[L] = prob_exp(em[(t - 1) * V + (c ? tok[j - 1] : 0)]);
        ++L;
        if (c) {
            --j;
            if (j == 0) { ok = 1; break; }
        }
    }
    if (!ok) return -1;
    for (int64_t a = 0, b = L - 1; a < b; ++a, --b) {
        int32_t x = ptok[a]; ptok[a] = ptok[b]; ptok[b] = x;
        x = ptime[a]; ptime[a] = ptime[b]; ptime[b] = x;
        float y = pprob[a]; pprob[a] = pprob[b]; pprob[b] = y;
    }
    return L;
}

/* alignment.py:438-454.  Score = Python left-to-right double sum / count. */
int64_t wxo_merge_repeats(const int32_t* ptok, const int32_t* ptime, const float* pprob, int64_t L,
                          int32_t* s_tok, int32_t* s_start, int32_t* s_end, double* s_score) {
    int64_t i1 = 0, i2 = 0, S = 0;
    while (i1 < L) {
        while (i2 < L && ptok[i1] == ptok[i2]) ++i2;
        double sum = 0.0;
        for (int64_t k = i1; k < i2; ++k) sum += (double)pprob[k];
        s_tok[S] = ptok[i1];
        s_start[S] = ptime[i1];
        s_end[S] = ptime[i2 - 1] + 1;
        s_score[S] = sum / (double)(i2 - i1);
        ++S;
        i1 = i2;
    }
    return S;
}

/* align()'s use of the three (alignment.py:242-250) without materialising anything the
 * caller does not need.  Outputs N token segments; returns 0, or -1 when backtrack fails.
 * Scratch: trellis (T+1)*(N+1) floats + 3*T path entries, allocated here. */
int wxo_align_dp(const float* em, int64_t T, int32_t V, const int32_t* tok, int64_t N, int32_t blank,
                 int32_t* seg_start, int32_t* seg_end, double* seg_score, int64_t* t_start_out) {
    float* tr = (float*)malloc(sizeof(float) * (size_t)(T + 1) * (size_t)(N + 1));
    int32_t* ptok = (int32_t*)malloc(sizeof(int32_t) * (size_t)(T + 1));
    int32_t* ptime = (int32_t*)malloc(sizeof(int32_t) * (size_t)(T + 1));
    float* pprob = (float*)malloc(sizeof(float) * (size_t)(T + 1));
    int32_t* stok = (int32_t*)malloc(sizeof(int32_t) * (size_t)(T + 1));
    int rc = -1;
    if (tr && ptok && ptime && pprob && stok) {
        wxo_trellis(em, T, V, tok, N, blank, tr);
        int64_t L = wxo_backtrack(tr, em, T, V, tok, N, blank, ptok, ptime, pprob, t_start_out);
        if (L >= 0) {
            wxo_merge_repeats(ptok, ptime, pprob, L, stok, seg_start, seg_end, seg_score);
            rc = 0;
        }
    }
    free(tr); free(ptok); free(ptime); free(pprob); free(stok);
    return rc;
}

/* ------------------------------------------------------------------ Binarize (vad.py:118-180)
 * One class column of F scores; pyannote timestamps ts[i] = middle of window i =
 * 0.5*(s + (s + duration)) with s = start + i*step (no FMA).  Thresholds compared in fp32
 * (NumPy 2 / NEP 50 weak-scalar promotion of the Python float threshold).  The region list
 * is what Annotation keeps: regions of length <= 1e-6 s are dropped (pyannote Segment
 * truthiness).  Returns region count, or -1 if cap is exceeded. */
static inline double sw_middle(double start, double step, double dur, int64_t i) {
    double s = start + (double)i * step;
    double e = s + dur;
    return 0.5 * (s + e);
}

static int emit_region(double a, double b, double* rs, double* re, int64_t* n, int64_t cap) {
    if (!((b - a) > 1e-6)) return 0;
    if (*n >= cap) return -1;
    rs[*n] = a; re[*n] = b; ++*n;
    return 0;
}

int64_t wxo_binarize(const float* y, int64_t F, double sw_start, double sw_step, double sw_dur,
                     float onset, float offset, double max_duration, double pad_onset, double pad_offset,
                     double* rs, double* re, int64_t cap) {
    int64_t n = 0;
    if (F <= 0) return 0;
    /* curr_scores / curr_timestamps as frame indices: [stale?] + frames lo..hi-1 */
    int64_t* buf = (int64_t*)malloc(sizeof(int64_t) * (size_t)(F + 1));
    if (!buf) return -2;
    int64_t blen = 0;
    double start = sw_middle(sw_start, sw_step, sw_dur, 0);
    int active = y[0] > onset;
    buf[blen++] = 0;
    double t = start;
    for (int64_t i = 1; i < F; ++i) {
        t = sw_middle(sw_start, sw_step, sw_dur, i);
        float yi = y[i];
        if (active) {
            if (t - start > max_duration) {
                int64_t sa = blen / 2;
                int64_t best = sa;
                float bv = y[buf[sa]];
                if (!isnan(bv)) {
                    for (int64_t k = sa + 1; k < blen; ++k) {
                        float v = y[buf[k]];
                        if (isnan(v)) { best = k; break; }
                        if (v < bv) { bv = v; best = k; }
                    }
                }
                double mt = sw_middle(sw_start, sw_step, sw_dur, buf[best]);
                if (emit_region(start - pad_onset, mt + pad_offset, rs, re, &n, cap)) { n = -1; break; }
                start = mt;
                memmove(buf, buf + best + 1, sizeof(int64_t) * (size_t)(blen - best - 1));
                blen -= best + 1;
            } else if (yi < offset) {
                if (emit_region(start - pad_onset, t + pad_offset, rs, re, &n, cap)) { n = -1; break; }
                start = t;
                active = 0;
                blen = 0;
            }
            buf[blen++] = i;
        } else if (yi > onset) {
            start = t;
            active = 1;
        }
    }
    if (n >= 0 && active) {
        if (emit_region(start - pad_onset, t + pad_offset, rs, re, &n, cap)) n = -1;
    }
    free(buf);
    return n;
}
