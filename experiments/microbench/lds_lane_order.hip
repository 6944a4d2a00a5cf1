// Does one ds_add_f32 whose active lanes share an LDS address apply them in ascending lane order?
// Each trial: random initial bins, random addresses (many collisions), random exec mask, values of
// mixed magnitude (order-sensitive float sums). The host folds every trial in ascending and in
// descending lane order and counts bit mismatches against the device. Contention variant: 8 waves per
// workgroup, each on its own LDS region, 256 workgroups.
// build: hipcc --offload-arch=gfx950 -O3 -o lds_lane_order lds_lane_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

#define NB 64  // bins per wave region
#define OPS 32 // ds_add instructions per trial

__global__ void k_order(const float* __restrict__ init, const int* __restrict__ addr, const float* __restrict__ val,
                        const unsigned long long* __restrict__ mask, float* __restrict__ out) {
    __shared__ float lds[8][NB];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int trial = blockIdx.x * 8 + wave;
    lds[wave][lane] = init[trial * NB + lane];
    __builtin_amdgcn_wave_barrier();
    for (int op = 0; op < OPS; ++op) {
        const size_t b = ((size_t)trial * OPS + op) * 64 + lane;
        if ((mask[(size_t)trial * OPS + op] >> lane) & 1ull) atomicAdd(&lds[wave][addr[b]], val[b]);
    }
    __builtin_amdgcn_wave_barrier();
    out[trial * NB + lane] = lds[wave][lane];
}

int main() {
    const int blocks = 256, trials = blocks * 8;
    std::mt19937 rng(7);
    std::vector<float> init((size_t)trials * NB), val((size_t)trials * OPS * 64), out((size_t)trials * NB);
    std::vector<int> addr((size_t)trials * OPS * 64);
    std::vector<unsigned long long> mask((size_t)trials * OPS);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& x : init) x = u(rng) * 1e3f;
    for (size_t i = 0; i < val.size(); ++i) {
        const int e = (int)(rng() % 40) - 20;
        val[i] = ldexpf(u(rng), e);
    }
    for (size_t t = 0; t < (size_t)trials * OPS; ++t) {
        const int kind = (int)(t % 4);
        const int span = kind == 0 ? 1 : kind == 1 ? 4 : kind == 2 ? 16 : 64;  // distinct addresses in play
        for (int l = 0; l < 64; ++l) addr[t * 64 + l] = (int)(rng() % span);
        unsigned long long m = ((unsigned long long)rng() << 32) | rng();
        if (t % 3 == 0) m = ~0ull;
        if (t % 5 == 0) m = 0x0FFFFFFFFFFFFFFFull;  // the apply's 60-lane pattern
        mask[t] = m;
    }
    float *d_init, *d_val, *d_out; int* d_addr; unsigned long long* d_mask;
    hipMalloc(&d_init, init.size() * 4); hipMalloc(&d_val, val.size() * 4); hipMalloc(&d_out, out.size() * 4);
    hipMalloc(&d_addr, addr.size() * 4); hipMalloc(&d_mask, mask.size() * 8);
    hipMemcpy(d_init, init.data(), init.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_val, val.data(), val.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_addr, addr.data(), addr.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_mask, mask.data(), mask.size() * 8, hipMemcpyHostToDevice);
    long long mis_up = 0, mis_down = 0, order_sensitive = 0;
    for (int rep = 0; rep < 20; ++rep) {
        k_order<<<blocks, 512>>>(d_init, d_addr, d_val, d_mask, d_out);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
        hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost);
        for (int t = 0; t < trials; ++t) {
            float up[NB], dn[NB];
            for (int j = 0; j < NB; ++j) up[j] = dn[j] = init[(size_t)t * NB + j];
            for (int op = 0; op < OPS; ++op) {
                const size_t base = ((size_t)t * OPS + op) * 64;
                const unsigned long long m = mask[(size_t)t * OPS + op];
                for (int l = 0; l < 64; ++l)
                    if ((m >> l) & 1ull) up[addr[base + l]] = up[addr[base + l]] + val[base + l];
                for (int l = 63; l >= 0; --l)
                    if ((m >> l) & 1ull) dn[addr[base + l]] = dn[addr[base + l]] + val[base + l];
            }
            for (int j = 0; j < NB; ++j) {
                const float g = out[(size_t)t * NB + j];
                unsigned a, b, c; memcpy(&a, &g, 4); memcpy(&b, &up[j], 4); memcpy(&c, &dn[j], 4);
                mis_up += a != b; mis_down += a != c;
                if (rep == 0) order_sensitive += b != c;
            }
        }
    }
    printf("{\"bins_checked\": %lld, \"order_sensitive_bins\": %lld, \"mismatch_ascending\": %lld, \"mismatch_descending\": %lld}\n",
           (long long)trials * NB * 20, order_sensitive, mis_up, mis_down);
    return 0;
}
