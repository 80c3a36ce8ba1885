// probe_duplex.hip — can the PCIe link run the HostMemory stage's upload and
// write-back at once (measurement tool, not product)?  Times, alone and
// together: the TX upload (one DMA copy host -> HBM), a DMA copy HBM -> host,
// and a kernel writing through the mapped host alias, dense or in the f1 C3
// pattern (1 M frames of 368 B at a 4-KiB stride, as image_writeback does).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// frames of `len` bytes at `stride`, 16 B per lane, a wave per frame
__global__ void scatter_write(const unsigned char* src, unsigned char* host, size_t nframes, unsigned len,
                              size_t stride) {
  const size_t nw = (size_t) gridDim.x * (blockDim.x / 64);
  const unsigned lane = threadIdx.x & 63u;
  for (size_t f = (size_t) blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; f < nframes; f += nw) {
    for (unsigned o = lane * 16u; o < len; o += 1024u) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(src + f * len + o);
      if (o + 16u <= len) *reinterpret_cast<u32x4*>(host + f * stride + o) = v;
      else
        for (unsigned b = 0; b < len - o; ++b) host[f * stride + o + b] = src[f * len + o + b];
    }
  }
}

int main(int argc, char** argv) {
  const size_t nframes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 20);
  const unsigned len = 368;
  const size_t stride = 4096, bytes = nframes * len;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned char *dA, *dB, *hA, *hB, *hS, *aS, *aB;
  CK(hipMalloc(&dA, bytes));
  CK(hipMalloc(&dB, bytes));
  CK(hipMemset(dB, 7, bytes));
  CK(hipHostMalloc(&hA, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hB, bytes, hipHostMallocMapped));
  CK(hipHostMalloc(&hS, nframes * stride, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&aS), hS, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&aB), hB, 0));
  for (size_t i = 0; i < bytes; i += 4096) hA[i] = 1;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2, f1, f2;
  for (hipEvent_t* e : {&e0, &e1, &e2, &f1, &f2}) CK(hipEventCreate(e));
  auto up = [&](hipStream_t s) { CK(hipMemcpyAsync(dA, hA, bytes, hipMemcpyHostToDevice, s)); };
  auto down_dma = [&](hipStream_t s) { CK(hipMemcpyAsync(hB, dB, bytes, hipMemcpyDeviceToHost, s)); };
  auto down_kernel = [&](hipStream_t s, int bpc) {
    hipLaunchKernelGGL(scatter_write, dim3(cus * bpc), dim3(256), 0, s, dB, aS, nframes, len, stride);
    CK(hipGetLastError());
  };
  auto down_dense = [&](hipStream_t s, int bpc) {
    hipLaunchKernelGGL(scatter_write, dim3(cus * bpc), dim3(256), 0, s, dB, aB, nframes, len, (size_t) len);
    CK(hipGetLastError());
  };
  auto report = [&](const char* what, hipEvent_t a, hipEvent_t b, hipEvent_t c, double n1, double n2) {
    float t1 = 0, t2 = 0;
    CK(hipEventElapsedTime(&t1, a, b));
    if (c) CK(hipEventElapsedTime(&t2, a, c));
    if (c)
      std::printf("{\"case\": \"%s\", \"ms_first\": %.3f, \"ms_second\": %.3f, \"GBps_first\": %.1f, \"GBps_second\": %.1f}\n",
                  what, t1, t2, n1 / t1 / 1e6, n2 / t2 / 1e6);
    else
      std::printf("{\"case\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f}\n", what, t1, n1 / t1 / 1e6);
  };
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    up(s1);
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    report("up_dma", e0, e1, nullptr, bytes, 0);

    CK(hipEventRecord(e0, s2));
    down_dma(s2);
    CK(hipEventRecord(e1, s2));
    CK(hipEventSynchronize(e1));
    report("down_dma", e0, e1, nullptr, bytes, 0);

    for (int bpc : {2, 8}) {
      CK(hipEventRecord(e0, s2));
      down_kernel(s2, bpc);
      CK(hipEventRecord(e1, s2));
      CK(hipEventSynchronize(e1));
      char name[64];
      std::snprintf(name, sizeof name, "down_kernel_4k_stride_bpc%d", bpc);
      report(name, e0, e1, nullptr, bytes, 0);
      CK(hipEventRecord(e0, s2));
      down_dense(s2, bpc);
      CK(hipEventRecord(e1, s2));
      CK(hipEventSynchronize(e1));
      std::snprintf(name, sizeof name, "down_kernel_dense_bpc%d", bpc);
      report(name, e0, e1, nullptr, bytes, 0);
    }

    // together: both start at e0
    CK(hipEventRecord(e0, s1));
    CK(hipStreamWaitEvent(s2, e0, 0));
    up(s1);
    down_dma(s2);
    CK(hipEventRecord(f1, s1));
    CK(hipEventRecord(f2, s2));
    CK(hipDeviceSynchronize());
    report("up_dma+down_dma", e0, f1, f2, bytes, bytes);

    for (int bpc : {2, 8}) {
      CK(hipEventRecord(e0, s1));
      CK(hipStreamWaitEvent(s2, e0, 0));
      up(s1);
      down_kernel(s2, bpc);
      CK(hipEventRecord(f1, s1));
      CK(hipEventRecord(f2, s2));
      CK(hipDeviceSynchronize());
      char name[64];
      std::snprintf(name, sizeof name, "up_dma+down_kernel_4k_bpc%d", bpc);
      report(name, e0, f1, f2, bytes, bytes);
    }
  }
  return 0;
}
