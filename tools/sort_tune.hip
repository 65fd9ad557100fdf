// sort_tune.hip -- times rocPRIM radix_sort_pairs configurations on the two sort
// shapes of the rasterizer (development tool, not part of the library):
//   depth: P = 1M, u32 keys (float bits), values = counting iterator, bits [0,32)
//   tile : R = 8M, u16 keys (tile id < 8160), values = counting iterator, bits [0,13)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sort_tune.hip -o tools/sort_tune
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include <rocprim/rocprim.hpp>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

template <class Cfg, class K>
float time_sort(const char* name, const K* keys_in, K* keys_out, uint32_t* vals_out, size_t n, unsigned end_bit,
                int iters = 20) {
    size_t bytes = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bytes, keys_in, keys_out, rocprim::counting_iterator<uint32_t>(0),
                                      vals_out, n, 0, end_bit));
    void* tmp;
    CK(hipMalloc(&tmp, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++)
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, keys_in, keys_out, rocprim::counting_iterator<uint32_t>(0),
                                          vals_out, n, 0, end_bit));
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; i++)
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, keys_in, keys_out, rocprim::counting_iterator<uint32_t>(0),
                                          vals_out, n, 0, end_bit));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-48s n=%9zu bits=%2u  %8.1f us\n", name, n, end_bit, ms / iters * 1e3);
    CK(hipFree(tmp));
    return ms / iters;
}

template <int BS, int IPT, int RB>
using OS = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                      rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                                                          rocprim::kernel_config<BS, IPT>, RB>,
                                      0>;
using DEF = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

int main() {
    std::mt19937 rng(0);
    // depth keys: float bits of z ~ U[2, 12] for 87%, 0xffffffff for the rest
    const size_t P = 1000000;
    std::vector<uint32_t> dk(P);
    std::uniform_real_distribution<float> uz(2.f, 12.f), u01(0.f, 1.f);
    for (auto& k : dk) {
        float z = uz(rng);
        memcpy(&k, &z, 4);
        if (u01(rng) > 0.87f) k = 0xffffffffu;
    }
    const size_t R = 7939550;
    std::vector<uint16_t> tk(R);
    std::uniform_int_distribution<int> ut(0, 8159);
    for (auto& k : tk) k = (uint16_t)ut(rng);

    uint32_t *d_dk, *d_dko, *d_v;
    uint16_t *d_tk, *d_tko;
    CK(hipMalloc(&d_dk, P * 4));
    CK(hipMalloc(&d_dko, P * 4));
    CK(hipMalloc(&d_v, R * 4));
    CK(hipMalloc(&d_tk, R * 2));
    CK(hipMalloc(&d_tko, R * 2));
    CK(hipMemcpy(d_dk, dk.data(), P * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tk, tk.data(), R * 2, hipMemcpyHostToDevice));

    time_sort<DEF>("depth default(onesweep)", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<256, 16, 11>>("depth os<256,16,rb11>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<512, 8, 11>>("depth os<512,8,rb11>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<256, 8, 11>>("depth os<256,8,rb11>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<256, 4, 11>>("depth os<256,4,rb11>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<1024, 4, 8>>("depth os<1024,4,rb8>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<256, 4, 8>>("depth os<256,4,rb8>", d_dk, d_dko, d_v, P, 32);
    time_sort<OS<128, 4, 8>>("depth os<128,4,rb8>", d_dk, d_dko, d_v, P, 32);

    time_sort<DEF>("tile default(onesweep)", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<256, 12, 7>>("tile os<256,12,rb7>", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<512, 16, 7>>("tile os<512,16,rb7>", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<256, 16, 13>>("tile os<256,16,rb13>", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<512, 16, 13>>("tile os<512,16,rb13>", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<1024, 8, 13>>("tile os<1024,8,rb13>", d_tk, d_tko, d_v, R, 13);
    time_sort<OS<512, 8, 11>>("tile os<512,8,rb11>", d_tk, d_tko, d_v, R, 13);
    // memcpy reference: bytes moved by one pass (read+write key+value)
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < 20; i++) CK(hipMemcpyAsync(d_v, d_v + R / 2, R / 2 * 4, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("d2d copy of %zu MB: %.1f us (%.0f GB/s r+w)\n", R / 2 * 4 >> 20, ms / 20 * 1e3, 2.0 * R / 2 * 4 / (ms / 20 * 1e-3) / 1e9);
    return 0;
}
