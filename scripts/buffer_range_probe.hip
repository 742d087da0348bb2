// buffer_range_probe.hip -- diagnostic: does a raw buffer load's range check (num_records) cover the
// SGPR offset (soffset) or only the lane's voffset?  Every address read lies inside one valid 1 MiB
// allocation filled with 1.0f; the descriptor's num_records is 4 KiB.
// build: hipcc --offload-arch=gfx950 -O2 scripts/buffer_range_probe.hip -o build/buffer_range_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_probe(const float *buf, float *out, unsigned soff, unsigned voff) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(buf), 0, 4096, 0x00020000);
    const unsigned lane = threadIdx.x;
    out[lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 4 * lane, soff, 0));
}

int main() {
    float *buf, *out;
    (void)hipMalloc(&buf, 1 << 20);
    (void)hipMalloc(&out, 256);
    float ones[1 << 18];
    for (auto &v : ones) v = 1.0f;
    (void)hipMemcpy(buf, ones, sizeof ones, hipMemcpyHostToDevice);
    const unsigned cases[][2] = {{0, 0}, {8192, 0}, {0, 8192}, {4000, 0}, {0, 4000}};
    for (const auto &c : cases) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, buf, out, c[0], c[1]);
        float h[64];
        (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
        int ones_read = 0;
        for (float v : h) ones_read += v == 1.0f;
        std::printf("soffset %5u voffset %5u (+4*lane): %2d of 64 lanes read data, %2d read 0\n", c[0], c[1], ones_read,
                    64 - ones_read);
    }
    return 0;
}
