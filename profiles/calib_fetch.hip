// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access pattern
// the step kernel uses on its state: one 8-byte element per lane, 13 SoA
// arrays read and written (dwordx2 loads/stores, fully coalesced).
// Known bytes: n * 8 * 13 read + n * 8 * 13 written per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void soa_rw(double **a, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int k = 0; k < 13; ++k) a[k][i] = a[k][i] * 1.0000001 + 1.0;
}
int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 24);   // 16 M doubles x 13 = 1.7 GB (beyond MALL)
    double *h[13];
    for (int k = 0; k < 13; ++k) { if (hipMalloc(&h[k], n * 8) != hipSuccess) return 1; hipMemset(h[k], 0, n * 8); }
    double **d;
    hipMalloc(&d, sizeof(h));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(soa_rw, dim3((n + 255) / 256), dim3(256), 0, 0, d, n);
    hipDeviceSynchronize();
    printf("calib bytes_read_per_launch=%lld bytes_written_per_launch=%lld\n", (long long)(n * 8 * 13),
           (long long)(n * 8 * 13));
    return 0;
}
