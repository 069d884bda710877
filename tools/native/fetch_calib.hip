// fetch_calib.hip — calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the walkers use (MI355X_MICROARCH.md, HBM section: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Every kernel touches a KNOWN number of distinct 128-B lines of an 8 GiB buffer that no
// earlier kernel touched since the last 1 GiB eviction sweep (Infinity Cache is 256 MiB), so
// the bytes that must come from HBM are known: lines x 128 B for the random kernels
// (one line per lane, lanes scattered by an odd multiplier mod 2^26 lines), the buffer size
// for the streaming ones.  tools/fetch_calib.py divides the counters by those figures.
//
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/native/fetch_calib tools/native/fetch_calib.hip
//   run:   rocprofv3 --pmc FETCH_SIZE -- tools/native/fetch_calib   (one counter group per pass)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

constexpr uint64_t kLines = 1ull << 26;  // 8 GiB of 128-B lines
constexpr uint64_t kBytes = kLines * 128ull;
constexpr uint32_t kMul = 2654435761u;  // odd: a bijection mod 2^26

__device__ __forceinline__ uint64_t line_of(uint32_t i, uint32_t salt) {
    return (uint64_t)((i * kMul + salt) & (uint32_t)(kLines - 1));
}

// One read of W bytes per lane at offset `off` of its own random line.
template <int W>
__global__ void rand_read(const uint8_t* __restrict__ buf, uint32_t n, uint32_t salt, uint32_t off,
                          uint32_t* __restrict__ sink) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = buf + line_of(i, salt) * 128ull + off;
    uint32_t v;
    if (W == 1) v = *p;
    else if (W == 4) v = *(const uint32_t*)p;
    else if (W == 8) { const uint2 q = *(const uint2*)p; v = q.x ^ q.y; }
    else { const uint4 q = *(const uint4*)p; v = q.x ^ q.y ^ q.z ^ q.w; }
    if (v == 77u) sink[i & 1023] = v;  // never true for the zeroed buffer; keeps the load
}

// Two 1-B reads per lane, one in each 64-B half of its line.
__global__ void rand_read_halves(const uint8_t* __restrict__ buf, uint32_t n, uint32_t salt,
                                 uint32_t* __restrict__ sink) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = buf + line_of(i, salt) * 128ull;
    const uint32_t v = p[5] + p[64 + 7];
    if (v == 77u) sink[i & 1023] = v;
}

// Coalesced 16 B per lane over `bytes` starting at `base`.
__global__ void stream_read(const uint4* __restrict__ buf, uint64_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n16; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 q = buf[j];
        acc ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

template <int W>
__global__ void rand_write(uint8_t* __restrict__ buf, uint32_t n, uint32_t salt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* p = buf + line_of(i, salt) * 128ull;
    if (W == 4) *(uint32_t*)p = i;
    else *(uint4*)p = make_uint4(i, i, i, i);
}

__global__ void stream_write(uint4* __restrict__ buf, uint64_t n16) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n16; j += (uint64_t)gridDim.x * blockDim.x)
        buf[j] = make_uint4((uint32_t)j, 0u, 0u, 0u);
}

int main() {
    uint8_t* buf = nullptr;
    uint8_t* evict = nullptr;
    uint32_t* sink = nullptr;
    const uint64_t kEvict = 1ull << 30;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&evict, kEvict));
    CK(hipMalloc(&sink, 4096 * sizeof(uint32_t)));
    CK(hipMemset(buf, 0, kBytes));
    CK(hipMemset(sink, 0, 4096 * sizeof(uint32_t)));
    CK(hipDeviceSynchronize());
    const uint32_t n = 1u << 22;  // lanes = distinct lines per random kernel (512 MiB of lines)
    const dim3 blk(256), grd((n + 255) / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto evict_l3 = [&]() {  // 1 GiB streamed write + read: nothing of the previous kernel stays in the 256 MiB L3
        hipLaunchKernelGGL(stream_write, dim3(4096), blk, 0, 0, (uint4*)evict, kEvict / 16);
        hipLaunchKernelGGL(stream_read, dim3(4096), blk, 0, 0, (const uint4*)evict, kEvict / 16, sink + 2048);
    };
    auto timed = [&](const char* name, double lines_bytes, auto launch) {
        evict_l3();
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-18s known_bytes %.0f  ms %.4f  GB/s(known) %.1f\n", name, lines_bytes, ms, lines_bytes / (ms * 1e6));
    };
    const double L = (double)n * 128.0;
    // salts keep the random kernels on different lines (n * kMul spreads; the salt shifts)
    timed("rand_read_1B", L, [&] { hipLaunchKernelGGL(rand_read<1>, grd, blk, 0, 0, buf, n, 0u, 3u, sink); });
    timed("rand_read_4B", L, [&] { hipLaunchKernelGGL(rand_read<4>, grd, blk, 0, 0, buf, n, 1u << 24, 8u, sink); });
    timed("rand_read_8B", L, [&] { hipLaunchKernelGGL(rand_read<8>, grd, blk, 0, 0, buf, n, 2u << 24, 16u, sink); });
    timed("rand_read_16B", L, [&] { hipLaunchKernelGGL(rand_read<16>, grd, blk, 0, 0, buf, n, 3u << 24, 32u, sink); });
    timed("rand_read_1B_hi", L, [&] { hipLaunchKernelGGL(rand_read<1>, grd, blk, 0, 0, buf, n, 1u << 23, 100u, sink); });
    timed("rand_read_halves", L, [&] { hipLaunchKernelGGL(rand_read_halves, grd, blk, 0, 0, buf, n, 3u << 23, sink); });
    timed("stream_read_16B", (double)(1ull << 30), [&] {
        hipLaunchKernelGGL(stream_read, dim3(8192), blk, 0, 0, (const uint4*)(buf + (4ull << 30)), (1ull << 30) / 16, sink);
    });
    timed("rand_write_4B", L, [&] { hipLaunchKernelGGL(rand_write<4>, grd, blk, 0, 0, buf, n, 5u << 22); });
    timed("rand_write_16B", L, [&] { hipLaunchKernelGGL(rand_write<16>, grd, blk, 0, 0, buf, n, 7u << 22); });
    timed("stream_write_16B", (double)(1ull << 30), [&] {
        hipLaunchKernelGGL(stream_write, dim3(8192), blk, 0, 0, (uint4*)(buf + (6ull << 30)), (1ull << 30) / 16);
    });
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    CK(hipFree(evict));
    CK(hipFree(sink));
    return 0;
}
