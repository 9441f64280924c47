// Step-latency micro-benchmark (development tool): cycles (s_memtime) per DP time step of
// one wave, for variants of the fused recurrence step of align_dp (one cell per lane):
//   c = left(cur) + et  (DPP wave_shr:1 fused into the add)
//   s = cur + eb
//   bit: word = 2 word + (c > s)
//   cur = maximum(s, c)
// The chain through `cur` is what paces a latency-bound launch; this measures how the
// decision bit and the hazard padding cost on it.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define R8(x) R4(x) R4(x)
// v0 cur, v1 s, v2 c, v3 word, v8 et, v9 eb, v4..v7 scratch
#define KER(NAME, BODY)                                                                                  \
    __global__ void NAME(unsigned long long* out, float* o) {                                            \
        __shared__ float sh[512];                                                                        \
        sh[threadIdx.x & 511] = 0.f;                                                                     \
        float x = threadIdx.x * 1e-3f;                                                                   \
        asm volatile(                                                                                    \
            "v_mov_b32 v0, %0\n v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, 0\n v_mov_b32 v4, %0\n" \
            " v_mov_b32 v5, %0\n v_mov_b32 v6, %0\n v_mov_b32 v7, %0\n v_mov_b32 v8, %0\n v_mov_b32 v9, %0\n" \
            " v_mov_b32 v10, 0\n s_mov_b32 m0, -1" ::"v"(x)                                              \
            : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "m0");                  \
        __syncthreads();                                                                                 \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                            \
        for (int i = 0; i < 64; ++i)                                                                     \
            asm volatile(BODY ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "vcc", \
                         "s20", "s21", "memory");                                                        \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                            \
        float r;                                                                                         \
        asm volatile("s_waitcnt lgkmcnt(0)\n v_add_f32 %0, v0, v3" : "=v"(r));                          \
        if ((threadIdx.x & 63) == 0) {                                                                   \
            out[2 * (threadIdx.x >> 6)] = t0;                                                            \
            out[2 * (threadIdx.x >> 6) + 1] = t1;                                                        \
        }                                                                                                \
        if (r == 1234.5f) o[0] = r;                                                                      \
    }

// current form: dpp-add, add, cmp/addc via VCC, maximum3, 2 wait states before the next DPP
KER(k_cur, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
               "v_add_f32 v1, v0, v9\n v_cmp_gt_f32 vcc, v2, v1\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
               "v_maximum3_f32 v0, v1, v2, v2\n s_nop 1\n"))
// same, the stay add placed between max and the DPP (one wait state less)
KER(k_cur2, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                "v_cmp_gt_f32 vcc, v2, v1\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
                "v_maximum3_f32 v0, v1, v2, v2\n v_add_f32 v1, v0, v9\n s_nop 0\n"))
// decision bit through an SGPR pair (e64 compare)
KER(k_sgpr, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                "v_add_f32 v1, v0, v9\n v_cmp_gt_f32_e64 s[20:21], v2, v1\n v_addc_co_u32_e64 v3, s[20:21], v3, v3, s[20:21]\n"
                "v_maximum3_f32 v0, v1, v2, v2\n s_nop 1\n"))
// decision bit without SGPRs: sign of s - c, shifted in with alignbit
KER(k_sub, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
               "v_add_f32 v1, v0, v9\n v_sub_f32 v4, v1, v2\n v_alignbit_b32 v3, v3, v4, 31\n"
               "v_maximum3_f32 v0, v1, v2, v2\n s_nop 1\n"))
// sub form with the stay add between max and DPP
KER(k_sub2, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                "v_sub_f32 v4, v1, v2\n v_maximum3_f32 v0, v1, v2, v2\n v_alignbit_b32 v3, v3, v4, 31\n"
                "v_add_f32 v1, v0, v9\n"))
// no decision bit (lower bound of the forward alone)
KER(k_nobit, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                 "v_add_f32 v1, v0, v9\n v_maximum3_f32 v0, v1, v2, v2\n s_nop 1\n"))
KER(k_nobit2, R16("v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                  "v_maximum3_f32 v0, v1, v2, v2\n v_add_f32 v1, v0, v9\n s_nop 0\n"))
// current form + the per-step LDS operand read kept two steps ahead (ds_read, partial wait)
KER(k_cur_lds, R16("ds_read_b32 v8, v10\n s_waitcnt lgkmcnt(1)\n"
                   "v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                   "v_add_f32 v1, v0, v9\n v_cmp_gt_f32 vcc, v2, v1\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
                   "v_maximum3_f32 v0, v1, v2, v2\n s_nop 1\n"))
KER(k_sub2_lds, R16("ds_read_b32 v8, v10\n s_waitcnt lgkmcnt(1)\n"
                    "v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                    "v_sub_f32 v4, v1, v2\n v_maximum3_f32 v0, v1, v2, v2\n v_alignbit_b32 v3, v3, v4, 31\n"
                    "v_add_f32 v1, v0, v9\n"))
// two cells per lane (C = 2): cell 1's change input is cell 0's old value (no DPP)
KER(k_c2, R16("v_add_f32_dpp v2, v5, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
              "v_add_f32 v6, v0, v8\n v_add_f32 v1, v0, v9\n v_add_f32 v7, v5, v9\n"
              "v_cmp_gt_f32 vcc, v2, v1\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
              "v_cmp_gt_f32 vcc, v6, v7\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n"
              "v_maximum3_f32 v0, v1, v2, v2\n v_maximum3_f32 v5, v7, v6, v6\n s_nop 1\n"))

// register-resident operands (the chunk's rows prefetched a chunk ahead: no wait in the step
// chain), one ds_read2_b32 of et and one of eb per two steps, best orders
#define STEP_CMP "v_add_f32 v1, v0, v9\n v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
                 "v_cmp_gt_f32 vcc, v2, v1\n v_maximum3_f32 v0, v1, v2, v2\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
#define STEP_SUB "v_add_f32 v1, v0, v9\n v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
                 "v_sub_f32 v4, v1, v2\n v_maximum3_f32 v0, v1, v2, v2\n v_alignbit_b32 v3, v3, v4, 31\n"
#define LDS2 "ds_read2_b32 v[12:13], v10 offset1:32\n ds_read2_b32 v[14:15], v10 offset0:64 offset1:96\n"
KER(k_reg_cmp, R8(LDS2 STEP_CMP STEP_CMP))
KER(k_reg_sub, R8(LDS2 STEP_SUB STEP_SUB))
KER(k_reg_cmp_nolds, R16(STEP_CMP))
KER(k_reg_sub_nolds, R16(STEP_SUB))
// the same with the DPP's old-value form (bound_ctrl off: lane 0 keeps the pre-added column-0
// change value in the destination)
#define STEP_SUB_OLD "v_add_f32 v1, v0, v9\n v_mov_b32 v2, v7\n v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                     "v_sub_f32 v4, v1, v2\n v_maximum3_f32 v0, v1, v2, v2\n v_alignbit_b32 v3, v3, v4, 31\n"
KER(k_reg_sub_old, R8(LDS2 STEP_SUB_OLD STEP_SUB_OLD))

int main() {
    unsigned long long* d;
    float* o;
    (void)hipMalloc(&d, 8 * 4096);
    (void)hipMalloc(&o, 64);
    struct {
        const char* n;
        void (*k)(unsigned long long*, float*);
    } ks[] = {{"cur (vcc bit)", k_cur},        {"cur, add before dpp", k_cur2}, {"sgpr-pair bit", k_sgpr},
              {"sub+alignbit bit", k_sub},     {"sub+alignbit, reordered", k_sub2}, {"no bit", k_nobit},
              {"no bit, reordered", k_nobit2}, {"cur + lds read", k_cur_lds}, {"sub reordered + lds", k_sub2_lds},
              {"C=2 cur", k_c2},
              {"reg cmp + ds_read2/2 steps", k_reg_cmp}, {"reg sub + ds_read2/2 steps", k_reg_sub},
              {"reg cmp, no lds", k_reg_cmp_nolds}, {"reg sub, no lds", k_reg_sub_nolds},
              {"reg sub, dpp old (+mov)", k_reg_sub_old}};
    for (int wps : {1, 2}) {
        printf("== %d wave(s) per SIMD (workgroup of %d waves on one CU)\n", wps, 4 * wps);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * 4 * wps), 0, 0, d, o);
            (void)hipDeviceSynchronize();
            unsigned long long h[64];
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * 4 * wps), 0, 0, d, o);
            (void)hipMemcpy(h, d, 8 * 2 * 4 * wps, hipMemcpyDeviceToHost);
            double sum = 0;
            for (int w = 0; w < 4 * wps; ++w) sum += (double)(h[2 * w + 1] - h[2 * w]);
            printf("  %-26s %6.2f cycles per step (wave-local)\n", k.n, sum / (4 * wps) / (64.0 * 16));
        }
    }
    return 0;
}
