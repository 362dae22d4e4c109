// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the fused env-step kernel.
//
// MI355X_MICROARCH.md (HBM / rocprofv3 section): on gfx950 FETCH_SIZE reports 1/2 of the bytes
// of a 16-B-per-lane streaming read; other access widths are uncalibrated. k_env_step_wave reads
// its per-env record with 4-B-per-lane loads on partial waves (lanes < 3, < 4, < 27, < 21) and
// its per-env scalars with one lane, so the x2 factor bench.py applies is an upper estimate
// there. This program replays those access patterns over a known byte count so the factor for
// each one can be read off a `rocprofv3 --pmc FETCH_SIZE` (and `--pmc WRITE_SIZE`) pass:
//   k_read16   16 B / lane streaming read of the records (the guide's calibrated case: x2)
//   k_read4    the wave kernel's record-load pattern, 4 B / lane on partial waves
//   k_read8s   one lane per env reads an 8-B scalar (progress / reset buffers)
//   k_readsec  4 lanes per env read the first 16 B of the record's last 128-B line only: the
//              fetch granularity (N * 128 if whole lines are fetched, N * 64 / N * 32 if sectors)
//   k_write4p  the record-store pattern without the sensors / pad (last line partly written):
//              its FETCH_SIZE shows whether the L2 fills a partly written line from HBM
//   k_write4   the wave kernel's record-store pattern, 4 B / lane on partial waves
//   k_write8s  one lane per env writes an 8-B scalar
//   k_code     no data traffic, 16384 straight-line FMAs (size: llvm-readelf on the code object): the instruction
//              fetch of a launch (every XCD's L2 fetches the code it runs once per launch)
// Every kernel runs one 64-lane wave per env, 4 envs per 256-thread workgroup, XCD-aware order.
// Known bytes per launch: records N * 384 (whole 128-B lines, every line of a record touched),
// scalars N * 8. Reads fold into a value that is stored only if it equals a sentinel the data
// never produces, so the read kernels write nothing.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -o run -- tools/fetch_calib N
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

constexpr int ES = 96;   // Humanoid record floats (pos 3, quat 4, vel 6, q 21, qd 21, eff 21, sens 12, pad)

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

// XCD-aware env order, as k_env_step_wave's wave_env(): workgroups are dealt round-robin to the
// 8 XCDs, so workgroup b takes env block (b % 8) * (G / 8) + b / 8 (each XCD one contiguous range)
__device__ __forceinline__ int env_id() {
    const unsigned G = gridDim.x, b = blockIdx.x;
    const int blk = (G & 7u) ? (int)b : (int)((b & 7u) * (G >> 3) + (b >> 3));
    return blk * 4 + (threadIdx.x >> 6);
}

__global__ __launch_bounds__(256) void k_read16(const float4* __restrict__ rec, int N, float* out) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N) return;
    float s = 0.0f;
    if (lane < ES / 4) { const float4 v = rec[(size_t)i * (ES / 4) + lane]; s = v.x + v.y + v.z + v.w; }
    if (s == -1234.5f) out[i] = s;
}

__global__ __launch_bounds__(256) void k_read4(const float* __restrict__ rec, int N, float* out) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N) return;
    const float* r = rec + (size_t)i * ES;
    float s = 0.0f;
    if (lane < 3) s += r[lane];                                   // root pos
    if (lane < 4) s += r[3 + lane];                               // root quat
    if (lane < 6) s += r[7 + lane];                               // root vel
    else if (lane < 27) s += r[34 + lane - 6];                    // qd
    if (lane < 21) s += r[13 + lane];                             // q
    if (lane < 21) s += r[55 + lane];                             // efforts (pre-step)
    if (s == -1234.5f) out[i] = s;
}

__global__ __launch_bounds__(256) void k_read8s(const int64_t* __restrict__ v, int N, float* out) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N || lane != 0) return;
    const int64_t x = v[i];
    if (x == -12345) out[i] = (float)x;
}

__global__ __launch_bounds__(256) void k_readsec(const float* __restrict__ rec, int N, float* out) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N) return;
    float s = 0.0f;
    if (lane < 4) s = rec[(size_t)i * ES + 64 + lane];
    if (s == -1234.5f) out[i] = s;
}

__global__ __launch_bounds__(256) void k_write4p(float* rec, int N) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N) return;
    float* r = rec + (size_t)i * ES;
    const float x = (float)lane;
    if (lane < 64) r[lane] = x;                                   // lines 0, 1 whole
    if (lane < 12) r[64 + lane] = x;                              // line 2: 48 of 128 B
}

__global__ __launch_bounds__(256) void k_write4(float* rec, int N) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N) return;
    float* r = rec + (size_t)i * ES;
    const float x = (float)lane;
    if (lane < 3) r[lane] = x;
    if (lane < 4) r[3 + lane] = x;
    if (lane < 6) r[7 + lane] = x;
    else if (lane < 27) r[34 + lane - 6] = x;
    if (lane < 21) r[13 + lane] = x;
    if (lane < 21) r[55 + lane] = x;
    if (lane < 12) r[76 + lane] = x;                              // sensors
    if (lane < 8) r[88 + lane] = x;                               // pad: every line written whole
}

__global__ __launch_bounds__(256) void k_write8s(int64_t* v, int N) {
    const int i = env_id(), lane = threadIdx.x & 63;
    if (i >= N || lane != 0) return;
    v[i] = i;
}

// straight-line body by macro expansion (a #pragma unroll of this size is left as a loop)
#define F1 x = __builtin_fmaf(x, a, b); asm volatile("" : "+v"(x));
#define F16 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1
#define F256 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16 F16
#define F4096 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256 F256
__global__ __launch_bounds__(256) void k_code(float a, float b, float* out) {
    float x = (float)threadIdx.x;
    F4096 F4096 F4096 F4096
    if (x == -1234.5f) out[0] = x;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    float *rec, *out;
    int64_t* sc;
    CK(hipMalloc(&rec, (size_t)N * ES * 4));
    CK(hipMalloc(&out, (size_t)N * 4));
    CK(hipMalloc(&sc, (size_t)N * 8));
    CK(hipMemset(rec, 0, (size_t)N * ES * 4));
    CK(hipMemset(sc, 0, (size_t)N * 8));
    const dim3 g((N + 3) / 4), b(256);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_read16, g, b, 0, 0, (const float4*)rec, N, out);
        hipLaunchKernelGGL(k_read4, g, b, 0, 0, rec, N, out);
        hipLaunchKernelGGL(k_read8s, g, b, 0, 0, sc, N, out);
        hipLaunchKernelGGL(k_write4, g, b, 0, 0, rec, N);
        hipLaunchKernelGGL(k_readsec, g, b, 0, 0, rec, N, out);
        hipLaunchKernelGGL(k_write4p, g, b, 0, 0, rec, N);
        hipLaunchKernelGGL(k_write8s, g, b, 0, 0, sc, N);
        hipLaunchKernelGGL(k_code, dim3(2048), b, 0, 0, 0.999f, 1e-3f, out);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("{\"N\": %d, \"reps\": %d, \"record_bytes\": %zu, \"scalar_bytes\": %zu}\n", N, reps,
           (size_t)N * ES * 4, (size_t)N * 8);
    CK(hipFree(rec)); CK(hipFree(out)); CK(hipFree(sc));
    return 0;
}
