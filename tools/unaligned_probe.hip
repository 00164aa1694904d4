// unaligned_probe.hip — does buffer_load_dwordx4 honour byte-unaligned
// offsets on this gfx950 box (SH_MEM_CONFIG alignment mode), and do
// buffer_store_byte stores land exactly?  Decides whether the per-object host
// path may run the GF pass on packed rows (pitch = shard size, any size).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t *src, uint8_t *dst, int n) {
    const int t = threadIdx.x;  // lane t loads 16 B at byte offset 16*t + 3
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, n, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, n, 0x00020000);
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, t * 16, 3, 2);
    if (t < 63) {
        __builtin_amdgcn_raw_buffer_store_b128(v, rd, t * 16, 5, 16);
    } else {  // last lane: bytes 0..6 only, one byte store each
        for (int b = 0; b < 7; ++b)
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[b / 4] >> (8 * (b % 4))), rd, t * 16 + b, 5, 16);
    }
}

int main() {
    const int n = 4096;
    uint8_t h[n], o[n];
    for (int i = 0; i < n; ++i) h[i] = (uint8_t)(i * 7 + 1);
    uint8_t *ds, *dd;
    if (hipMalloc(&ds, n) || hipMalloc(&dd, n)) return 1;
    (void)hipMemcpy(ds, h, n, hipMemcpyHostToDevice);
    (void)hipMemset(dd, 0xEE, n);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, ds, dd, n);
    if (hipDeviceSynchronize()) return 2;
    (void)hipMemcpy(o, dd, n, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        uint8_t want = 0xEE;
        const int j = i - 5;  // dst byte i holds src byte j + 3 for j in [0, 63*16 + 7)
        if (j >= 0 && j < 63 * 16 + 7) want = h[j + 3];
        if (o[i] != want) {
            if (bad < 5) std::printf("byte %d: got %02x want %02x\n", i, o[i], want);
            ++bad;
        }
    }
    std::printf("unaligned b128 loads/stores + byte tail stores: %s (%d bad bytes)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 3 : 0;
}
