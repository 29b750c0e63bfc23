// Calibration probe (tuning only): how much does VALU work beside v_mfma_f32_32x32x2_f32 cost on
// gfx950? One workgroup per CU of W waves (W = 4: 1 wave per SIMD, W = 8: 2), each wave runs
// STEPS steps of 4 MFMAs on 4 independent accumulators with random operands, plus V independent
// VALU ops (v_max_i32 via inline asm, exact count) per MFMA. Prints achieved MFMA TFLOP/s and the
// cycles per MFMA per SIMD at an assumed 2.4 GHz.
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_valu_probe.hip -o build/mfma_valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int STEPS = 2048;

template <int V>
__device__ __forceinline__ void filler(int (&r)[8], int y) {
#pragma unroll
    for (int k = 0; k < V; ++k) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r[k & 7]) : "v"(y));
}

template <int V>
__global__ void probe(const float* in, float* out) {
    const int tid = threadIdx.x;
    float a0 = in[tid & 255], a1 = in[(tid + 17) & 255], b0 = in[(tid + 33) & 255],
          b1 = in[(tid + 71) & 255];
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    int r[8];
    for (int k = 0; k < 8; ++k) r[k] = tid * (k + 3);
    const int y = tid ^ 0x55;
    for (int s = 0; s < STEPS; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
        filler<V>(r, y);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
        filler<V>(r, y);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
        filler<V>(r, y);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
        filler<V>(r, y);
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int e = 0; e < 16; ++e) s += acc[i][e];
    for (int k = 0; k < 8; ++k) s += (float)r[k];
    out[blockIdx.x * blockDim.x + tid] = s;
}

template <int V>
void run(int waves, const float* in, float* out) {
    const int blocks = 256, threads = waves * 64;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(threads), 0, 0, in, out);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(threads), 0, 0, in, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / reps;
    const double mfma_per_simd = (double)waves / 4 * STEPS * 4;
    const double flop = 256.0 * waves * STEPS * 4 * 4096;
    printf("{\"waves_per_cu\": %d, \"valu_per_mfma\": %d, \"us\": %.2f, \"TFs\": %.1f, "
           "\"cyc_per_mfma_at_2.4GHz\": %.1f}\n",
           waves, V, us, flop / us / 1e6, us * 2400.0 / mfma_per_simd);
}


// The weight-gradient tile loop's structure, piece by piece (MODE): 1 = operands from register
// vectors P[i][e] / Q[j][e] (16 steps x 4 MFMAs per tile); 2 = + the tile's 8 operand MFMAs;
// 3 = + the mask / relu VALU of finish(); 4 = 3 with ping-pong buffers one tile ahead.
template <int MODE>
__global__ void tile_probe(const float* in, float* out, int tiles) {
    const int tid = threadIdx.x, lane = tid & 63;
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    f32x16 P[2], Q[2], Pn[2], Qn[2];
    for (int i = 0; i < 2; ++i)
        for (int e = 0; e < 16; ++e) {
            P[i][e] = in[(lane + e + i) & 255];
            Q[i][e] = in[(lane + 3 * e + 7 * i) & 255];
        }
    float g = in[lane], w0 = in[lane + 1], w1 = in[lane + 2], x0 = in[lane + 3], x1 = in[lane + 4];
    uint32_t m0 = 0x5a5a ^ lane, m1 = 0x3c3c ^ lane;
    const f32x16 zero = {};
    auto issue = [&](f32x16 (&Pd)[2], f32x16 (&Qd)[2]) {
        for (int i = 0; i < 2; ++i) {
            Pd[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(g, w0, zero, 0, 0, 0);
            Qd[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1, g, zero, 0, 0, 0);
        }
        for (int i = 0; i < 2; ++i) Qd[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, w1, Qd[i], 0, 0, 0);
        for (int i = 0; i < 2; ++i) Qd[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, w0, Qd[i], 0, 0, 0);
    };
    auto finish = [&](f32x16 (&Pd)[2], f32x16 (&Qd)[2]) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            Pd[0][e] = __int_as_float(__float_as_int(Pd[0][e]) & __builtin_amdgcn_sbfe((int)m0, e, 1));
            Pd[1][e] = __int_as_float(__float_as_int(Pd[1][e]) & __builtin_amdgcn_sbfe((int)m1, e, 1));
            Qd[0][e] = __int_as_float(max(__float_as_int(Qd[0][e]), 0));
            Qd[1][e] = __int_as_float(max(__float_as_int(Qd[1][e]), 0));
        }
    };
    auto body = [&](f32x16 (&Pc)[2], f32x16 (&Qc)[2], f32x16 (&Pd)[2], f32x16 (&Qd)[2]) {
        if (MODE >= 4) issue(Pd, Qd);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(Pc[0][e], Qc[0][e], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(Pc[0][e], Qc[1][e], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(Pc[1][e], Qc[0][e], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(Pc[1][e], Qc[1][e], acc[1][1], 0, 0, 0);
        }
        if (MODE >= 4) finish(Pd, Qd);
        m0 = m0 * 1664525u + 1013904223u;
        m1 = m1 * 22695477u + 1u;
    };
    for (int t = 0; t < tiles; t += 2) {
        if (MODE == 2 || MODE == 3) issue(P, Q);
        if (MODE == 3) finish(P, Q);
        body(P, Q, Pn, Qn);
        if (MODE == 2 || MODE == 3) issue(P, Q);
        if (MODE == 3) finish(P, Q);
        body(MODE >= 4 ? Pn : P, MODE >= 4 ? Qn : Q, P, Q);
    }
    float s = 0.f;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int e = 0; e < 16; ++e) s += acc[i][j][e];
    out[blockIdx.x * blockDim.x + tid] = s;
}

template <int MODE>
void run_tile(const float* in, float* out) {
    const int blocks = 256, threads = 512, tiles = 512;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(tile_probe<MODE>, dim3(blocks), dim3(threads), 0, 0, in, out, tiles);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(tile_probe<MODE>, dim3(blocks), dim3(threads), 0, 0, in, out, tiles);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / reps;
    const double useful = 2.0 * tiles * 64;  // wgrad MFMAs per SIMD (2 waves)
    printf("{\"tile_mode\": %d, \"us\": %.2f, \"cyc_per_wgrad_mfma_at_2.4GHz\": %.1f}\n", MODE, us,
           us * 2400.0 / useful);
}

int main() {
    float *in, *out;
    hipMalloc(&in, 256 * sizeof(float));
    hipMalloc(&out, 256 * 1024 * sizeof(float));
    float h[256];
    unsigned s = 12345;
    for (int i = 0; i < 256; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
    }
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    run_tile<1>(in, out);
    run_tile<2>(in, out);
    run_tile<3>(in, out);
    run_tile<4>(in, out);
    for (int w : {4, 8}) {
        run<0>(w, in, out);
        run<2>(w, in, out);
        run<4>(w, in, out);
        run<8>(w, in, out);
        run<12>(w, in, out);
        run<16>(w, in, out);
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
