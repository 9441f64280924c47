// VALU throughput micro-benchmark (development tool): SIMD cycles per wave-instruction with
// 4 waves per SIMD (one 1024-thread workgroup on one CU), 8 independent chains per wave, for
// the candidate forms of the DP step's decision bit and adds.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R2(x) x x
#define R4(x) x x x x
#define CLOB "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", \
             "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "vcc"
#define KER(NAME, BODY)                                                                                     \
    __global__ void __launch_bounds__(1024) NAME(unsigned long long* out, float* o) {                       \
        float x = threadIdx.x * 1e-3f;                                                                      \
        asm volatile(                                                                                       \
            "v_mov_b32 v0, %0\n v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, %0\n v_mov_b32 v4, %0\n"    \
            " v_mov_b32 v5, %0\n v_mov_b32 v6, %0\n v_mov_b32 v7, %0\n v_mov_b32 v8, %0\n v_mov_b32 v9, %0\n"  \
            " v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, 0\n v_mov_b32 v13, 0\n"                  \
            " v_mov_b32 v14, 0\n v_mov_b32 v15, 0\n v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n"                    \
            " v_mov_b32 v18, 0\n v_mov_b32 v19, 0\n v_mov_b32 v20, %0\n v_mov_b32 v21, %0\n"                  \
            " v_mov_b32 v22, %0\n v_mov_b32 v23, %0\n v_mov_b32 v24, %0\n v_mov_b32 v25, %0" ::"v"(x)         \
            : CLOB);                                                                                        \
        __syncthreads();                                                                                    \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < 64; ++i) asm volatile(BODY ::: CLOB);                                          \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                               \
        float r;                                                                                            \
        asm volatile("v_add_f32 %0, v0, v12\n v_add_f32 %0, %0, v1" : "=v"(r));                             \
        if ((threadIdx.x & 63) == 0) {                                                                      \
            out[2 * (threadIdx.x >> 6)] = t0;                                                               \
            out[2 * (threadIdx.x >> 6) + 1] = t1;                                                           \
        }                                                                                                   \
        if (r == 1234.5f) o[0] = r;                                                                         \
    }
// 8 independent instructions per body, repeated 4x -> 32 instructions per iteration
#define I8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)
#define ADD(i) "v_add_f32 v" #i ", v" #i ", v20\n"
#define SUB(i) "v_sub_f32 v" #i ", v20, v" #i "\n"
#define MAX(i) "v_max_f32 v" #i ", v" #i ", v20\n"
#define MAX3(i) "v_maximum3_f32 v" #i ", v" #i ", v20, v20\n"
#define ALIGN(i) "v_alignbit_b32 v1" #i ", v1" #i ", v" #i ", 31\n"
#define CMPC(i) "v_cmp_gt_f32 vcc, v" #i ", v20\n v_addc_co_u32 v1" #i ", vcc, v1" #i ", v1" #i ", vcc\n"
#define LSHLADD(i) "v_lshl_add_u32 v1" #i ", v1" #i ", 1, v" #i "\n"
#define ADDU(i) "v_add_u32 v1" #i ", v1" #i ", v" #i "\n"
#define LSHR(i) "v_lshrrev_b32 v1" #i ", 31, v" #i "\n"
#define CNDM(i) "v_cmp_gt_f32 vcc, v" #i ", v20\n v_cndmask_b32 v1" #i ", v1" #i ", v20, vcc\n"
// one cell of the step, current form: s, c, cmp+addc, maximum3 (5 instr); cells i use v(i) cur,
// v(1i) word; scratch v21 (s), v22 (c)
#define STEP_CUR(i) "v_add_f32 v21, v" #i ", v20\n v_add_f32 v22, v" #i ", v23\n v_cmp_gt_f32 vcc, v22, v21\n" \
                    " v_addc_co_u32 v1" #i ", vcc, v1" #i ", v1" #i ", vcc\n v_maximum3_f32 v" #i ", v21, v22, v22\n"
// sub + alignbit form (5 instr): d = s - c, word = (word << 1) | sign(d)... sign(s-c) = (c > s)
#define STEP_SUB(i) "v_add_f32 v21, v" #i ", v20\n v_add_f32 v22, v" #i ", v23\n v_sub_f32 v24, v21, v22\n" \
                    " v_alignbit_b32 v1" #i ", v1" #i ", v24, 31\n v_maximum3_f32 v" #i ", v21, v22, v22\n"
KER(k_add, R4(I8(ADD)))
KER(k_sub, R4(I8(SUB)))
KER(k_max, R4(I8(MAX)))
KER(k_max3, R4(I8(MAX3)))
KER(k_align, R4(I8(ALIGN)))
KER(k_cmpc, R2(I8(CMPC)))
#define PK(a, b) "v_pk_add_f32 v[" #a ":" #b "], v[" #a ":" #b "], v[20:21]\n"
#define PK8 PK(0, 1) PK(2, 3) PK(4, 5) PK(6, 7) PK(8, 9) PK(10, 11) PK(12, 13) PK(14, 15)
KER(k_pkadd, R4(PK8))
KER(k_lshladd, R4(I8(LSHLADD)))
KER(k_addu, R4(I8(ADDU)))
KER(k_lshr, R4(I8(LSHR)))
KER(k_cndm, R2(I8(CNDM)))
KER(k_step_cur, I8(STEP_CUR))
KER(k_step_sub, I8(STEP_SUB))

// NaN signs the hardware produces: x[0] = +inf, x[1] = -inf, x[2] = -NaN (0xffc00000),
// x[3] = 1
__global__ void k_nan(const float* x, unsigned* r) {
    float a = x[0], b = x[1], n = x[2], one = x[3], v;
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(v) : "v"(a), "v"(a));  // inf - inf
    r[0] = __float_as_uint(v);
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(v) : "v"(a), "v"(b));  // inf + -inf
    r[1] = __float_as_uint(v);
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(v) : "v"(one), "v"(n));  // 1 - (-nan)
    r[2] = __float_as_uint(v);
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(v) : "v"(n), "v"(one));  // -nan + 1
    r[3] = __float_as_uint(v);
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(v) : "v"(b), "v"(b));  // -inf - -inf
    r[4] = __float_as_uint(v);
}

int main() {
    {
        float hx[4] = {__builtin_inff(), -__builtin_inff(), __builtin_bit_cast(float, 0xffc00000u), 1.f};
        float* dx;
        unsigned* dr;
        unsigned hr[5];
        (void)hipMalloc(&dx, 16);
        (void)hipMalloc(&dr, 20);
        (void)hipMemcpy(dx, hx, 16, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_nan, dim3(1), dim3(1), 0, 0, dx, dr);
        (void)hipMemcpy(hr, dr, 20, hipMemcpyDeviceToHost);
        printf("inf-inf %08x  inf+-inf %08x  1-(-nan) %08x  -nan+1 %08x  -inf-(-inf) %08x\n", hr[0], hr[1], hr[2],
               hr[3], hr[4]);
    }
    unsigned long long* d;
    float* o;
    (void)hipMalloc(&d, 8 * 4096);
    (void)hipMalloc(&o, 64);
    struct {
        const char* n;
        void (*k)(unsigned long long*, float*);
        int per;  // instructions per loop iteration
    } ks[] = {{"v_add_f32", k_add, 32},          {"v_sub_f32", k_sub, 32},         {"v_max_f32", k_max, 32},
              {"v_maximum3_f32", k_max3, 32},    {"v_alignbit_b32", k_align, 32},  {"cmp+addc (per pair)", k_cmpc, 16},
              {"v_pk_add_f32", k_pkadd, 32},     {"v_lshl_add_u32", k_lshladd, 32}, {"v_add_u32", k_addu, 32},
              {"v_lshrrev_b32", k_lshr, 32},     {"cmp+cndmask (pair)", k_cndm, 16}, {"step cur (per cell)", k_step_cur, 8},
              {"step sub (per cell)", k_step_sub, 8}};
    for (int wps : {1, 2, 4}) {
        printf("== %d wave(s) per SIMD\n", wps);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(256 * wps), 0, 0, d, o);
            (void)hipDeviceSynchronize();
            unsigned long long h[64];
            hipLaunchKernelGGL(k.k, dim3(1), dim3(256 * wps), 0, 0, d, o);
            (void)hipMemcpy(h, d, 8 * 2 * 4 * wps, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            for (int w = 0; w < 4 * wps; ++w) {
                lo = h[2 * w] < lo ? h[2 * w] : lo;
                hi = h[2 * w + 1] > hi ? h[2 * w + 1] : hi;
            }
            const double simd = (double)(hi - lo) / (64.0 * k.per * wps);
            printf("  %-24s %5.2f SIMD cycles per wave-instruction\n", k.n, simd);
        }
    }
    return 0;
}
