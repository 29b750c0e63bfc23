// Throughput probe for the weight-gradient inner loop shape on gfx950: one 256-thread block per
// CU, each wave runs STEPS steps of 4 independent v_mfma_f32_32x32x2_f32 (4 accumulators), with
// the A/B operands either re-read from LDS every step (ds_read2 as in k_wgrad) or kept in
// registers. Prints achieved TFLOP/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int STEPS = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out) {
    __shared__ float lds[2 * 32 * 132];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    for (int i = tid; i < 2 * 32 * 132; i += 256) lds[i] = 0.001f * (i & 7);
    __syncthreads();
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const float* pw = lds + h * 132 + l32;
    const float* qw = lds + 32 * 132 + h * 132 + l32;
    float a0 = pw[0], a1 = pw[32], b0 = qw[0], b1 = qw[32];
    for (int s = 0; s < STEPS; ++s) {
        float a0n = a0, a1n = a1, b0n = b0, b1n = b1;
        if (MODE == 0) {  // k_wgrad: next step's operands from LDS
            const int o = 2 * ((s + 1) & 15) * 132;
            a0n = pw[o]; a1n = pw[o + 32]; b0n = qw[o]; b1n = qw[o + 32];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a0n; a1 = a1n; b0 = b0n; b1 = b1n;
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int e = 0; e < 16; ++e) s += acc[i][e];
    out[blockIdx.x * 256 + tid] = s;
}

// same work as 16x16x4 (4x the instructions, 32 cycles each), 8 accumulators
template <int MODE>
__global__ __launch_bounds__(256) void probe16(float* out) {
    __shared__ float lds[2 * 32 * 132];
    const int tid = threadIdx.x;
    for (int i = tid; i < 2 * 32 * 132; i += 256) lds[i] = 0.001f * (i & 7);
    __syncthreads();
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* p = lds + (tid & 63);
    float a[4], b[4];
    for (int i = 0; i < 4; ++i) { a[i] = p[i * 64]; b[i] = p[2048 + i * 64]; }
    for (int s = 0; s < STEPS; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i * 4 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i * 4 + j], 0, 0, 0);
        if (MODE == 0) {
            const int o = ((s + 1) & 7) * 256;
            for (int i = 0; i < 4; ++i) { a[i] = p[o + i * 64]; b[i] = p[o + 2048 + i * 64]; }
        }
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + tid] = s;
}

template <typename K>
void run(const char* name, K k, int blocks, double flop_per_wave_step, float* out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double t = ms / 5 * 1e-3;
    const double fl = flop_per_wave_step * STEPS * blocks * 4;
    printf("%-28s blocks %4d  %8.1f us  %6.1f TF/s\n", name, blocks, t * 1e6, fl / t / 1e12);
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * 256 * 4);
    for (int blocks : {256, 512}) {
        run("32x32x2 lds-operands", probe<0>, blocks, 4 * 4096.0, out);
        run("32x32x2 reg-operands", probe<1>, blocks, 4 * 4096.0, out);
        run("16x16x4 lds-operands", probe16<0>, blocks, 16 * 2048.0, out);
        run("16x16x4 reg-operands", probe16<1>, blocks, 16 * 2048.0, out);
    }
    return 0;
}
