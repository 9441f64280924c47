// Step-latency micro-benchmark, part 2 (development tool): a register-resident DP step with
// 16-byte LDS operand loads, the column-0 helper's fp64 chain, and the two sharing SIMDs.
// Waves 0-3 run BODY_A (one per SIMD), waves 4-7 BODY_B (one more per SIMD) when present.
// hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R8(x) R4(x) R4(x)
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define CLOB "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", \
             "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29",  \
             "v30", "v31", "v32", "v33", "v34", "v35", "vcc", "memory"
#define KER2(NAME, BODY_A, BODY_B)                                                                          \
    __global__ void NAME(unsigned long long* out, float* o) {                                               \
        __shared__ float sh[1024];                                                                          \
        sh[threadIdx.x & 1023] = 1e-3f * (threadIdx.x & 7);                                                 \
        __syncthreads();                                                                                    \
        float x = threadIdx.x * 1e-3f;                                                                      \
        asm volatile(                                                                                       \
            "v_mov_b32 v0, %0\n v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, 0\n v_mov_b32 v4, %0\n"    \
            " v_mov_b32 v8, %0\n v_mov_b32 v9, %0\n v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n"                   \
            " v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n" ::"v"(x)          \
            : CLOB);                                                                                        \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                               \
        if (threadIdx.x < 256) {                                                                            \
            for (int i = 0; i < 64; ++i) asm volatile(BODY_A ::: CLOB);                                    \
        } else {                                                                                            \
            for (int i = 0; i < 64; ++i) asm volatile(BODY_B ::: CLOB);                                    \
        }                                                                                                   \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                               \
        float r;                                                                                            \
        asm volatile("s_waitcnt lgkmcnt(0)\n v_add_f32 %0, v0, v3\n v_add_f32 %0, %0, v20" : "=v"(r));     \
        if ((threadIdx.x & 63) == 0) {                                                                      \
            out[2 * (threadIdx.x >> 6)] = t0;                                                               \
            out[2 * (threadIdx.x >> 6) + 1] = t1;                                                           \
        }                                                                                                   \
        if (r == 1234.5f) o[0] = r;                                                                         \
    }

// DP step, cmp form (best order), operands in registers
#define STEP_CMP "v_add_f32 v1, v0, v9\n v_add_f32_dpp v2, v0, v8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
                 "v_cmp_gt_f32 vcc, v2, v1\n v_maximum3_f32 v0, v1, v2, v2\n v_addc_co_u32 v3, vcc, v3, v3, vcc\n"
// 16 steps with two ds_read_b128 per 4 steps (et, eb), none waited
#define DP_B128 R4("ds_read_b128 v[12:15], v10\n ds_read_b128 v[16:19], v11 offset:16\n" STEP_CMP STEP_CMP STEP_CMP STEP_CMP)
// 16 steps with three (et, eb, column-0 pre)
#define DP_B128x3 R4("ds_read_b128 v[12:15], v10\n ds_read_b128 v[16:19], v11 offset:16\n ds_read_b128 v[24:27], v11 offset:32\n" \
                     STEP_CMP STEP_CMP STEP_CMP STEP_CMP)
#define DP_NOLDS R16(STEP_CMP)
// bare dependent fp64 chain: 16 rows
#define F64_CHAIN R16("v_add_f64 v[20:21], v[20:21], v[22:23]\n")
// column-0 helper: 16 rows = 4 x (two broadcast b128 loads of em[.,0] and em[.,tok0] for 4
// rows, waited one group late; per row cvt in, fp64 add (the chain), cvt out, fp32 pre-add;
// one b128 store of the 4 pre values)
#define HROW(I) "v_cvt_f64_f32 v[22:23], v" #I "\n v_add_f64 v[20:21], v[20:21], v[22:23]\n v_cvt_f32_f64 v33, v[20:21]\n v_add_f32 v" #I ", v33, v" #I "\n"
#define HELPER R4("s_waitcnt lgkmcnt(2)\n" HROW(24) HROW(25) HROW(26) HROW(27) "ds_write_b128 v11, v[24:27] offset:512\n" \
                  "ds_read_b128 v[24:27], v11\n ds_read_b128 v[28:31], v11 offset:16\n")
// a stager-like light wave: one LDS op and a few SALU per 4 rows
#define LIGHT R4("s_add_u32 s20, s20, 1\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n")
#define IDLE "s_sleep 2\n"

KER2(k_dp_nolds, DP_NOLDS, IDLE)
KER2(k_dp_b128, DP_B128, IDLE)
KER2(k_dp_b128x3, DP_B128x3, IDLE)
KER2(k_chain, F64_CHAIN, IDLE)
KER2(k_helper, HELPER, IDLE)
KER2(k_dp_vs_helper, DP_B128, HELPER)
KER2(k_dp_vs_dp, DP_B128, DP_B128)
KER2(k_dp_vs_light, DP_B128, LIGHT)

int main() {
    unsigned long long* d;
    float* o;
    (void)hipMalloc(&d, 8 * 4096);
    (void)hipMalloc(&o, 64);
    struct {
        const char* n;
        void (*k)(unsigned long long*, float*);
        int waves;
    } ks[] = {{"DP reg, no lds", k_dp_nolds, 4},
              {"DP reg + 2 b128 / 4 steps", k_dp_b128, 4},
              {"DP reg + 3 b128 / 4 steps", k_dp_b128x3, 4},
              {"fp64 add chain (per add)", k_chain, 4},
              {"col-0 helper (per row)", k_helper, 4},
              {"DP b128 | helper on 2nd wave", k_dp_vs_helper, 8},
              {"DP b128 | DP b128 2nd wave", k_dp_vs_dp, 8},
              {"DP b128 | light 2nd wave", k_dp_vs_light, 8}};
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * k.waves), 0, 0, d, o);
        (void)hipDeviceSynchronize();
        unsigned long long h[64];
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * k.waves), 0, 0, d, o);
        (void)hipMemcpy(h, d, 8 * 2 * k.waves, hipMemcpyDeviceToHost);
        double a = 0, b = 0;
        for (int w = 0; w < 4; ++w) a += (double)(h[2 * w + 1] - h[2 * w]);
        for (int w = 4; w < k.waves; ++w) b += (double)(h[2 * w + 1] - h[2 * w]);
        printf("  %-30s waves 0-3: %6.2f cycles per step/row", k.n, a / 4 / (64.0 * 16));
        if (k.waves > 4) printf("   waves 4-7: %6.2f", b / 4 / (64.0 * 16));
        printf("\n");
    }
    return 0;
}
