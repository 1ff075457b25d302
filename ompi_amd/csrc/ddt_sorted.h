// ddt_sorted.h -- address-ordered two-pass plan of a large single-element index list
// (ddt_sorted.hip).  Internal to libddt_hip.so.
#pragma once

#include <cstdint>
#include <mutex>
#include <vector>

#include <hip/hip_runtime.h>

namespace ddt {

struct SortedList {
    uint32_t n = 0;          // blocks (one element each)
    uint32_t esz = 0;        // element bytes: 4, 8 or 16
    uint32_t ch = 0;         // elements per chunk (address order): rg / cdiv
    uint32_t rg = 0;         // elements per bucket (packed order): a 128 KiB LDS image
    uint32_t cdiv = 1;       // 2: half-size chunks, two pass-1 workgroups per CU
    uint32_t seg = 0;        // elements per segment of U
    uint32_t segb = 64;      // segment bytes: 64 or 128
    bool unpadded = false;   // runs packed end to end in U (segb = the lanes per run only)
    uint32_t nc = 0, nb = 0; // chunks, buckets
    uint32_t skew = 0;       // U slots between consecutive buckets (r6: buckets of exactly RG slots
                             // start 128 KiB apart, so one chunk's runs all fell on one DRAM
                             // channel; `ddt_tune sskew` bytes, read at build)
    uint32_t cst = 0;        // chunk-major U: elements from one chunk image to the next (ch + skew)
    uint64_t slots = 0;      // U slots, runs padded to whole segments
    uint64_t dev_bytes = 0;  // device bytes held (tables + U)
    uint32_t *A = nullptr;       // [n] element offset (units of esz) of the j-th block in address order
                                 // (freed after the build when the compressed form below fits)
    uint16_t *A16 = nullptr;     // [n] A[j] - Abase[j / 64]: 16-bit offsets inside 64-element groups
    uint32_t *Abase = nullptr;   // [n / 64] A of each group's first element
    uint16_t *SL = nullptr;      // [n] LDS slot of the j-th block inside its chunk
    uint16_t *off16 = nullptr;   // [nc][nb] LDS offset of run (c, k): exclusive prefix over k of
                                 // the blocks of chunk c whose packed position is in bucket k
    uint32_t *ub = nullptr;      // [nc][nb] first U slot of run (c, k); U is bucket-major
    uint32_t *bstart = nullptr;  // [nb + 1] first U slot of bucket k (k skews in); bucket k ends
                                 // at bstart[k + 1] - skew
    uint16_t *upos = nullptr;    // [slots] position inside its bucket, 0xFFFF = padding
    // chunk-major U (r6, `ddt_tune slayout`): a direction may keep U as the chunk images end to
    // end instead, so pass 1 / 1' streams its image and pass 2 / 2' reads / writes the runs
    // scattered; per bucket, the runs' U element offsets and their first slots within the bucket
    uint32_t *physT = nullptr;   // [nb][nc] c * cst + off(c, k)   (unpadded plans with nc <= 4096)
    uint16_t *vrelT = nullptr;   // [nb][nc] first slot of run (c, k) inside bucket k
                                 // in aligned quads, run by run)
    void *U = nullptr;           // [slots] scratch elements
    hipEvent_t done = nullptr;   // recorded after every run (U reuse across streams)
    hipStream_t last_stream = nullptr;
    bool used = false;
    std::mutex mu;               // run() from several host threads: one launch sequence at a time
    ~SortedList();
    // hand the tables and U to `out` (the plan releases them behind its stream fences)
    void take_blocks(std::vector<void *> &out);
    bool build(const int32_t *disp, uint32_t n, uint32_t esz, uint64_t span_elems, uint32_t segb,
               hipStream_t stream, uint32_t cdiv = 1, uint32_t skew_bytes = 0);
    // pol: access policy bits (POL_* in ddt_sorted.hip; ddt_tune "spol")
    // unroll: elements per thread in flight in pack 1's address-ordered gather (4, 8 or 16)
    // k2: the same for unpack pass 2' (4, 8 or 16)
    hipError_t run(uint8_t *user, uint8_t *packed, int dir, uint32_t pol, hipStream_t stream,
                   uint32_t unroll = 16, uint32_t k2 = 8);
};

}  // namespace ddt
