// MFMA verdict for the Delassus block of the articulated substep:
// A[r][s] = J_r . W_s for the R constraint rows of one env (J, W: R x nv, nv = 27 for Humanoid),
// built by one wavefront per env as the PGS set-up needs it: lane r ends up holding row r
// (A[r][0..R)). Three builds of the same block, each timed over many envs with HIP events:
//   valu  — the wave kernel's scheme (csrc/mi_wave.hpp, Delassus-space PGS set-up): lane r keeps
//           J_r in registers, W rows are LDS broadcasts, R x nv FMAs per lane;
//   mfma16 — v_mfma_f32_16x16x4f32 (R <= 16): 7 MFMAs over K = 28, then the 16 x 16 result
//           moved to lane = row (A is symmetric: column c of the MFMA output is row c) with
//           ds_bpermute;
//   mfma32 — v_mfma_f32_32x32x2f32 (R <= 32): 14 MFMAs, then the two lane halves exchange
//           their row halves.
// Build/run (GPU box): hipcc -O3 --offload-arch=gfx950 tools/mfma_delassus.hip -o /tmp/mfd && /tmp/mfd
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NV = 27, KP = 28, RM = 32, REPS = 64;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

// J, W of env i: [RM][KP] each (row-major, k padded to 28 with zeros). out[i][r] = sum_s A[r][s] * (s + 1)
// over the rows the lane holds (a checksum that needs every entry of row r).
__device__ void stage(const float* g, float* s) {
    for (int q = threadIdx.x; q < 2 * RM * KP; q += 64) s[q] = g[q];
    __syncthreads();
}

__global__ __launch_bounds__(64) void k_valu(const float* __restrict__ JW, float* out, int R) {
    __shared__ float sm[2 * RM * KP];
    const int i = blockIdx.x, lane = threadIdx.x;
    stage(JW + (size_t)i * 2 * RM * KP, sm);
    const float* sJ = sm;
    const float* sW = sm + RM * KP;
    float acc = 0.0f;
    for (int rep = 0; rep < REPS; ++rep) {
        asm volatile("" : "+v"(acc));
        const int rl = lane < R ? lane : 0;
        float Jr[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) Jr[c] = sJ[rl * KP + c];
        float Ar[RM];
#pragma unroll
        for (int s = 0; s < RM; ++s) {
            float a = 0.0f;
            if (s < R) {
                const float* w = sW + s * KP;
#pragma unroll
                for (int c = 0; c < NV; ++c) a += Jr[c] * w[c];
            }
            Ar[s] = a;
        }
#pragma unroll
        for (int s = 0; s < RM; ++s) acc += Ar[s] * (float)(s + 1);
    }
    if (lane < R) out[(size_t)i * RM + lane] = acc / REPS;
}

__global__ __launch_bounds__(64) void k_mfma16(const float* __restrict__ JW, float* out, int R) {
    __shared__ float sm[2 * RM * KP];
    const int i = blockIdx.x, lane = threadIdx.x;
    stage(JW + (size_t)i * 2 * RM * KP, sm);
    const float* sJ = sm;
    const float* sW = sm + RM * KP;
    float acc = 0.0f;
    const int row = lane & 15, kq = lane >> 4;
    for (int rep = 0; rep < REPS; ++rep) {
        asm volatile("" : "+v"(acc));
        v4f c = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k0 = 0; k0 < KP; k0 += 4) {
            const float a = sJ[row * KP + k0 + kq];     // A: J[row][k], lane = row + 16 k
            const float b = sW[row * KP + k0 + kq];     // B: W^T[k][col], lane = col + 16 k
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
        }
        // c[j] of lane l = A[4 (l / 16) + j][l % 16] = A[l % 16][4 (l / 16) + j] (symmetric):
        // lane l % 16 = r collects row r's 16 entries from lanes r, r + 16, r + 32, r + 48
        float Ar[16];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) Ar[4 * g + j] = __shfl(c[j], row + 16 * g);
#pragma unroll
        for (int s = 0; s < 16; ++s) acc += Ar[s] * (float)(s + 1);
    }
    if (lane < R) out[(size_t)i * RM + lane] = acc / REPS;
}

__global__ __launch_bounds__(64) void k_mfma32(const float* __restrict__ JW, float* out, int R) {
    __shared__ float sm[2 * RM * KP];
    const int i = blockIdx.x, lane = threadIdx.x;
    stage(JW + (size_t)i * 2 * RM * KP, sm);
    const float* sJ = sm;
    const float* sW = sm + RM * KP;
    float acc = 0.0f;
    const int row = lane & 31, kh = lane >> 5;
    for (int rep = 0; rep < REPS; ++rep) {
        asm volatile("" : "+v"(acc));
        v16f c = {};
#pragma unroll
        for (int k0 = 0; k0 < KP; k0 += 2) {
            const float a = sJ[row * KP + k0 + kh];
            const float b = sW[row * KP + k0 + kh];
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
        }
        // c[4 q + j] of lane l = A[8 q + 4 (l / 32) + j][l % 32] = row l % 32's entries
        // {8 q + 4 (l / 32) + j}; the partner lane l ^ 32 holds the other half
        float Ar[32];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float mine = c[4 * q + j];
                const float other = __shfl_xor(mine, 32);
                Ar[8 * q + 4 * kh + j] = mine;
                Ar[8 * q + 4 * (1 - kh) + j] = other;
            }
#pragma unroll
        for (int s = 0; s < 32; ++s) acc += Ar[s] * (float)(s + 1);
    }
    if (lane < R) out[(size_t)i * RM + lane] = acc / REPS;
}

int main() {
    const int E = 16384;   // envs (one wave each): 4 resident rounds at 16 waves / CU
    std::vector<float> h((size_t)E * 2 * RM * KP, 0.0f);
    srand(1);
    for (int e = 0; e < E; ++e) {
        float* J = &h[(size_t)e * 2 * RM * KP];
        float* W = J + RM * KP;
        for (int r = 0; r < RM; ++r)
            for (int k = 0; k < NV; ++k) {
                J[r * KP + k] = (float)rand() / RAND_MAX - 0.5f;
                W[r * KP + k] = (float)rand() / RAND_MAX - 0.5f;
            }
        // symmetric A like a Delassus block: W = J M^-1 with M = I here -> W = J
        for (int r = 0; r < RM; ++r)
            for (int k = 0; k < NV; ++k) W[r * KP + k] = J[r * KP + k];
    }
    float *dJW, *o1, *o2;
    CHECK(hipMalloc(&dJW, h.size() * 4));
    CHECK(hipMalloc(&o1, (size_t)E * RM * 4));
    CHECK(hipMalloc(&o2, (size_t)E * RM * 4));
    CHECK(hipMemcpy(dJW, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](auto kern, int R, float* o) {
        hipLaunchKernelGGL(kern, dim3(E), dim3(64), 0, 0, dJW, o, R);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int t = 0; t < 5; ++t) hipLaunchKernelGGL(kern, dim3(E), dim3(64), 0, 0, dJW, o, R);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms / 5;
    };
    // empty-rep baseline: staging alone (R = 0 rows computed by the VALU kernel)
    std::vector<float> r1((size_t)E * RM), r2((size_t)E * RM);
    printf("{\"envs\": %d, \"reps_per_env\": %d, \"nv\": %d, \"results\": [\n", E, REPS, NV);
    const int Rs[] = {8, 12, 16, 24, 32};
    bool first = true;
    for (int R : Rs) {
        const float tv = timeit(k_valu, R, o1);
        CHECK(hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost));
        float tm = 0.0f;
        const char* which = R <= 16 ? "mfma16" : "mfma32";
        tm = R <= 16 ? timeit(k_mfma16, R, o2) : timeit(k_mfma32, R, o2);
        CHECK(hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost));
        float t32 = timeit(k_mfma32, R, o2);
        double maxrel = 0.0;
        // checksums differ only by the row entries beyond R (zero in valu, real in mfma: the
        // MFMA tile always holds 16 / 32 rows); compare on the valid rows with R rows of J
        // zeroed beyond R is not possible here, so report the R = 16 / 32 cases' agreement
        if (R == 16 || R == 32) {
            std::vector<float> r3((size_t)E * RM);
            CHECK(hipMemcpy(r3.data(), o2, r3.size() * 4, hipMemcpyDeviceToHost));
            for (size_t q = 0; q < (size_t)E * RM; ++q) {
                if ((int)(q % RM) >= R) continue;
                const double ref = r1[q], got = (R == 16 ? r2[q] : r3[q]);
                const double d = fabs(ref - got) / (fabs(ref) + 1e-3);
                if (d > maxrel) maxrel = d;
            }
        }
        const double per_v = tv * 1e6 / ((double)E * REPS), per_m = tm * 1e6 / ((double)E * REPS);
        printf("%s {\"rows\": %d, \"valu_ns_per_block\": %.3f, \"%s_ns_per_block\": %.3f, \"mfma32_ns_per_block\": %.3f, "
               "\"valu_ms\": %.4f, \"mfma_ms\": %.4f, \"max_rel_diff\": %.2e}\n", first ? "" : ",", R, per_v, which, per_m,
               t32 * 1e6 / ((double)E * REPS), tv, tm, maxrel);
        first = false;
    }
    printf("]}\n");
    return 0;
}
