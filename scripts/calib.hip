// calib.hip -- calibration of the rocprofv3 memory counters on the engine's own access patterns
// (MI355X_MICROARCH.md "HBM": FETCH_SIZE is exact for no pattern but a
// 16-B-per-lane streaming read, where it reads half; other widths "calibrate on a known byte
// count in your own access pattern").  Not part of the product.
//
// Every pattern runs over a known set of lines, COLD (after a 1 GiB plain read that evicts the L2s
// and the Infinity Cache, dirty lines included; the flush is its own dispatch, `cal_flush`) and
// WARM (the same launch again at once).  Kernel names carry the pattern and the run (<P, 0> cold, <P, 1> warm), so one
// rocprofv3 --pmc pass per counter group yields per-dispatch counts; scripts/calibrate.py divides
// them by the known element / line counts.  Without the profiler the program prints its own
// event timings (JSON, one line per pattern and run).
//
// Patterns (L lines of 128 B; "sparse" = one line per 2 KiB, the x face's pitch):
//   0 stream_read     16-B/lane non-temporal loads of L*128 contiguous bytes (the guide's case)
//   1 stream_write    16-B/lane stores of L*128 contiguous bytes
//   2 gather8         one 8-B load per sparse line, written compactly (the x-face pack)
//   3 gather4         one 4-B load per sparse line (cfg3's dim-2 face)
//   4 gather8_pair64  two 8-B loads per sparse line, 64 B apart (does a line cost two 64-B halves?)
//   5 gather8_pair8   two adjacent 8-B loads per sparse line (same 64-B half)
//   6 scatter8_nt     one non-temporal 8-B store per sparse line (the x-face unpack)
//   7 scatter8        one plain 8-B store per sparse line
//   8 scatter4_nt     one non-temporal 4-B store per sparse line
//   9 gather8_dense   one 8-B load per line, lines adjacent (128-B pitch)
//  10 gather8_nt      pattern 2 with non-temporal loads
//  11 coop8           8 lanes per sparse line, each a 16-B load of its part (the whole line is
//                     read, like a stream); the lane holding the element writes it compactly
//  12 coop8_nt        pattern 11 with non-temporal loads
//  13 gather16        one 16-B load per sparse line (the element's 16-B part), 8 B written
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NPAT = 14;
constexpr const char *kNames[NPAT] = {"stream_read", "stream_write", "gather8", "gather4", "gather8_pair64",
                                      "gather8_pair8", "scatter8_nt", "scatter8", "scatter4_nt", "gather8_dense",
                                      "gather8_nt", "coop8", "coop8_nt", "gather16"};
constexpr size_t PITCH = 2048;

// plain (allocating) loads: the 1 GiB read displaces every line of the L2s and the Infinity
// Cache, dirty ones written back during the flush -- the next pattern starts cold AND clean
__global__ __launch_bounds__(256) void cal_flush(const u32x4 *__restrict__ p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const u32x4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u)
        sink[threadIdx.x] = acc;
}

// one thread per line (streams: one 16-B unit per thread)
template <int P, int RUN>
__global__ __launch_bounds__(256) void cal(uint8_t *__restrict__ big, uint8_t *__restrict__ compact, size_t L,
                                           uint32_t *sink)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (P == 0 || P == 1) {
        if (t >= L * 8)
            return;
        u32x4 *q = reinterpret_cast<u32x4 *>(big) + t;
        if (P == 0) {
            const u32x4 v = __builtin_nontemporal_load(q);
            if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u)
                sink[threadIdx.x] = v.x;
        } else {
            *q = u32x4{uint32_t(t), 1u, 2u, 3u};
        }
        return;
    }
    if (P == 11 || P == 12) {
        if (t >= L * 8)
            return;
        const size_t ln = t >> 3, part = t & 7;
        const u32x4 *q = reinterpret_cast<const u32x4 *>(big + ln * PITCH) + part;
        const u32x4 v = P == 12 ? __builtin_nontemporal_load(q) : *q;
        if (part == 0)
            reinterpret_cast<uint64_t *>(compact)[ln] = uint64_t(v.x) | (uint64_t(v.y) << 32);
        return;
    }
    if (t >= L)
        return;
    uint8_t *line = big + t * (P == 9 ? 128 : PITCH);
    uint64_t *c8 = reinterpret_cast<uint64_t *>(compact);
    switch (P) {
    case 2:
    case 9:
        c8[t] = *reinterpret_cast<const uint64_t *>(line);
        break;
    case 3:
        reinterpret_cast<uint32_t *>(compact)[t] = *reinterpret_cast<const uint32_t *>(line);
        break;
    case 4:
        c8[2 * t] = *reinterpret_cast<const uint64_t *>(line);
        c8[2 * t + 1] = *reinterpret_cast<const uint64_t *>(line + 64);
        break;
    case 5:
        c8[2 * t] = *reinterpret_cast<const uint64_t *>(line);
        c8[2 * t + 1] = *reinterpret_cast<const uint64_t *>(line + 8);
        break;
    case 6:
        __builtin_nontemporal_store(uint64_t(t) * 3 + RUN, reinterpret_cast<uint64_t *>(line));
        break;
    case 7:
        *reinterpret_cast<uint64_t *>(line) = uint64_t(t) * 3 + RUN;
        break;
    case 8:
        __builtin_nontemporal_store(uint32_t(t) * 3 + RUN, reinterpret_cast<uint32_t *>(line));
        break;
    case 10:
        c8[t] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(line));
        break;
    case 13: {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(line);
        c8[t] = uint64_t(v.x) | (uint64_t(v.y) << 32);
        break;
    }
    default:
        break;
    }
}

template <int P, int RUN>
void launch(uint8_t *big, uint8_t *compact, size_t L, uint32_t *sink)
{
    const size_t threads = (P == 0 || P == 1 || P == 11 || P == 12) ? L * 8 : L;
    hipLaunchKernelGGL((cal<P, RUN>), dim3(uint32_t((threads + 255) / 256)), dim3(256), 0, nullptr, big, compact, L,
                       sink);
}

template <int P>
void run_pattern(uint8_t *big, uint8_t *compact, size_t L, const u32x4 *flush, size_t nflush, uint32_t *sink,
                 hipEvent_t *ev, float *ms)
{
    hipLaunchKernelGGL(cal_flush, dim3(4096), dim3(256), 0, nullptr, flush, nflush, sink);
    CHK(hipEventRecord(ev[0], nullptr));
    launch<P, 0>(big, compact, L, sink);
    CHK(hipEventRecord(ev[1], nullptr));
    launch<P, 1>(big, compact, L, sink);
    CHK(hipEventRecord(ev[2], nullptr));
    CHK(hipEventSynchronize(ev[2]));
    CHK(hipEventElapsedTime(&ms[0], ev[0], ev[1]));
    CHK(hipEventElapsedTime(&ms[1], ev[1], ev[2]));
}

int main(int argc, char **argv)
{
    // L: lines per pattern (default 4 Mi: 512 MiB of lines, an 8 GiB span at the sparse pitch,
    // both beyond the 256 MiB Infinity Cache; 1 Mi: 128 MiB of lines, within it when warm)
    const size_t L = argc > 1 ? size_t(std::atol(argv[1])) : (size_t(4) << 20);
    const size_t span = L * PITCH;
    uint8_t *big = nullptr, *compact = nullptr;
    u32x4 *flush = nullptr;
    uint32_t *sink = nullptr;
    const size_t nflush = (size_t(1) << 30) / 16;
    CHK(hipMalloc(&big, span));
    CHK(hipMalloc(&compact, L * 16));
    CHK(hipMalloc(&flush, nflush * 16));
    CHK(hipMalloc(&sink, 1024));
    CHK(hipMemset(big, 1, span));
    CHK(hipMemset(flush, 2, nflush * 16));
    CHK(hipDeviceSynchronize());
    hipEvent_t ev[3];
    for (auto &e : ev)
        CHK(hipEventCreate(&e));
    float ms[NPAT][2];
    run_pattern<0>(big, compact, L, flush, nflush, sink, ev, ms[0]);
    run_pattern<1>(big, compact, L, flush, nflush, sink, ev, ms[1]);
    run_pattern<2>(big, compact, L, flush, nflush, sink, ev, ms[2]);
    run_pattern<3>(big, compact, L, flush, nflush, sink, ev, ms[3]);
    run_pattern<4>(big, compact, L, flush, nflush, sink, ev, ms[4]);
    run_pattern<5>(big, compact, L, flush, nflush, sink, ev, ms[5]);
    run_pattern<6>(big, compact, L, flush, nflush, sink, ev, ms[6]);
    run_pattern<7>(big, compact, L, flush, nflush, sink, ev, ms[7]);
    run_pattern<8>(big, compact, L, flush, nflush, sink, ev, ms[8]);
    run_pattern<9>(big, compact, L, flush, nflush, sink, ev, ms[9]);
    run_pattern<10>(big, compact, L, flush, nflush, sink, ev, ms[10]);
    run_pattern<11>(big, compact, L, flush, nflush, sink, ev, ms[11]);
    run_pattern<12>(big, compact, L, flush, nflush, sink, ev, ms[12]);
    run_pattern<13>(big, compact, L, flush, nflush, sink, ev, ms[13]);
    CHK(hipDeviceSynchronize());
    for (int p = 0; p < NPAT; ++p)
        for (int r = 0; r < 2; ++r)
            std::printf("{\"pattern\": \"%s\", \"id\": %d, \"run\": \"%s\", \"lines\": %zu, \"us\": %.2f}\n", kNames[p],
                        p, r ? "warm" : "cold", L, ms[p][r] * 1e3);
    return 0;
}
