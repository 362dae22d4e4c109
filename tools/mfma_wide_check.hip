// Stand-alone check of the wide Delassus MFMA set-up's data path (mi_pair.hpp MI_PAIR_WIDE_MFMA):
// one wave stores J^T to a global scratch through a buffer resource, reads it back in the
// v_mfma_f32_16x16x4f32 A-operand layout (other lanes' values), multiplies by W, stores the tiles
// and reads them back lane = row. Modes: 0 as in the kernel (wavefront fence only), 1 s_waitcnt on
// every counter after the stores, 2 an agent-scope acquire fence (L1 invalidate) after them.
// "prime" first loads the J^T lines so that stale copies sit in the vector L1 before the stores.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_wide_check.hip -o tools/mfma_wide_check
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NV = 27, KP = 28, KC = 7;

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void k_check(const float* J, const float* W, float* scr, float* out, int nrh,
                                             int mode, int prime) {
    const int l64 = threadIdx.x;
    float Jr[NV];
    for (int c = 0; c < NV; ++c) Jr[c] = J[l64 * NV + c];
    const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(scr, (short)0, 96 * 64 * 4, 0x00020000);
    const int avo = l64 * 4;
    float junk = 0.0f;
    if (prime) {
        for (int c = 0; c < KP; ++c)
            junk += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, avo, (64 + c) * 256, 0));
        for (int s = 0; s < 64; ++s)
            junk += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, avo, s * 256, 0));
    }
    for (int c = 0; c < KP; ++c) {
        const float jv = (c < NV && l64 < nrh) ? Jr[c] : 0.0f;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, jv), ars, avo, (64 + c) * 256, 0);
    }
    if (mode == 1) __builtin_amdgcn_s_waitcnt(0);
    if (mode == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wsync();
    const int lr = l64 & 15, lk = l64 >> 4;
    const int jvo = ((64 + lk) * 64 + lr) * 4;
    const int dvo = (4 * lk * 64 + lr) * 4;
#pragma unroll
    for (int S = 0; S < 4; ++S) {
        const int s = 16 * S + lr;
        float wb[KC];
#pragma unroll
        for (int K = 0; K < KC; ++K) {
            const int c = 4 * K + lk;
            wb[K] = (s < nrh && c < NV) ? W[s * NV + c] : 0.0f;
        }
#pragma unroll
        for (int R = 0; R < 4; ++R) {
            if (16 * R < nrh) {
                f4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int K = 0; K < KC; ++K) {
                    const float ja = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, jvo, (K * 256 + 16 * R) * 4, 0));
                    d = __builtin_amdgcn_mfma_f32_16x16x4f32(ja, wb[K], d, 0, 0, 0);
                }
                // the four D registers moved to VGPRs first: stored straight from the AGPR tuple,
                // this compiler emits four stores of a0 (ROCm 7.2 LLVM)
                float o4[4] = {d.x, d.y, d.z, d.w};
                asm volatile("" : "+v"(o4[0]), "+v"(o4[1]), "+v"(o4[2]), "+v"(o4[3]));
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o4[q]), ars, dvo, ((16 * R + q) * 64 + 16 * S) * 4, 0);
            }
        }
    }
    if (mode == 1) __builtin_amdgcn_s_waitcnt(0);
    if (mode == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wsync();
    for (int s = 0; s < 64; ++s)
        out[l64 * 64 + s] = s < nrh ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, avo, s * 256, 0)) : 0.0f;
    if (junk == 12345.678f) out[0] = junk;
}

int main() {
    std::vector<float> J(64 * NV), W(64 * NV);
    srand(7);
    for (auto& x : J) x = (float)rand() / RAND_MAX - 0.5f;
    for (auto& x : W) x = (float)rand() / RAND_MAX - 0.5f;
    float *dJ, *dW, *dS, *dO;
    hipMalloc(&dJ, J.size() * 4); hipMalloc(&dW, W.size() * 4);
    hipMalloc(&dS, 96 * 64 * 4); hipMalloc(&dO, 64 * 64 * 4);
    hipMemcpy(dJ, J.data(), J.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> o(64 * 64);
    for (int nrh : {51, 64, 33})
        for (int prime = 0; prime < 2; ++prime)
            for (int mode = 0; mode < 3; ++mode) {
                std::vector<float> junk(96 * 64, 777.0f);
                hipMemcpy(dS, junk.data(), junk.size() * 4, hipMemcpyHostToDevice);
                hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, dJ, dW, dS, dO, nrh, mode, prime);
                if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
                hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
                double maxerr = 0.0;
                int bad = 0, br = -1, bs = -1;
                for (int r = 0; r < nrh; ++r)
                    for (int s = 0; s < nrh; ++s) {
                        double ref = 0.0;   // out[r][s] = row s at lane r = J_s . W_r
                        for (int c = 0; c < NV; ++c) ref += (double)J[s * NV + c] * W[r * NV + c];
                        const double e = std::fabs(ref - o[r * 64 + s]);
                        if (e > maxerr) maxerr = e;
                        if (e > 1e-4 && bad++ == 0) { br = r; bs = s; }
                    }
                if (nrh == 64 && prime == 0 && mode == 0) {
                    FILE* f = fopen("gpurun_out/mfma_wide_dump.bin", "wb");
                    if (f) { fwrite(J.data(), 4, J.size(), f); fwrite(W.data(), 4, W.size(), f); fwrite(o.data(), 4, o.size(), f); fclose(f); }
                }
                printf("{\"nrh\": %d, \"prime\": %d, \"mode\": %d, \"max_err\": %.3g, \"bad\": %d, \"first_bad\": [%d, %d]}\n",
                       nrh, prime, mode, maxerr, bad, br, bs);
            }
    return 0;
}
