// probe_hostreg.hip — what hipHostRegister does with ranges that are not page
// aligned and share pages with other heap blocks (measurement tool, not
// product): exact-range registration, a second registration of another range
// on the same pages, copies of the unregistered neighbours, unregistering one
// while the other is in use, and device reads of the mapped alias.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define SHOW(x)                                                                        \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    std::printf("%-60s -> %d %s\n", #x, (int) e_, hipGetErrorString(e_));             \
    (void) hipGetLastError();                                                          \
  } while (0)

__global__ void sum_kernel(const unsigned char* p, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  atomicAdd(out, s);
}

static unsigned dev_sum(const void* alias, size_t n) {
  unsigned* d = nullptr;
  (void) hipMalloc(&d, 4);
  (void) hipMemset(d, 0, 4);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, static_cast<const unsigned char*>(alias), n, d);
  unsigned h = 0;
  hipError_t e = hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) std::printf("  dev_sum copy: %s\n", hipGetErrorString(e));
  (void) hipFree(d);
  return h;
}

int main() {
  // small heap blocks, adjacent: N1 | A | N2 | B | N3
  std::vector<unsigned char>* n1 = new std::vector<unsigned char>(1000, 1);
  std::vector<unsigned char>* a = new std::vector<unsigned char>(3000, 2);
  std::vector<unsigned char>* n2 = new std::vector<unsigned char>(1000, 3);
  std::vector<unsigned char>* b = new std::vector<unsigned char>(2000, 4);
  std::vector<unsigned char>* n3 = new std::vector<unsigned char>(1000, 5);
  std::printf("n1 %p a %p n2 %p b %p n3 %p (page offsets a %lu b %lu)\n", (void*) n1->data(), (void*) a->data(),
              (void*) n2->data(), (void*) b->data(), (void*) n3->data(),
              (unsigned long) ((uintptr_t) a->data() & 4095), (unsigned long) ((uintptr_t) b->data() & 4095));
  SHOW(hipHostRegister(a->data(), a->size(), hipHostRegisterMapped));
  void* da = nullptr;
  SHOW(hipHostGetDevicePointer(&da, a->data(), 0));
  std::printf("  alias a %p, device sum %u (want %u)\n", da, da ? dev_sum(da, a->size()) : 0u, 2u * 3000u);
  SHOW(hipHostRegister(a->data(), a->size(), hipHostRegisterMapped));  // same range again
  SHOW(hipHostRegister(b->data(), b->size(), hipHostRegisterMapped));  // another range, maybe same pages
  void* db = nullptr;
  SHOW(hipHostGetDevicePointer(&db, b->data(), 0));
  std::printf("  alias b %p, device sum %u (want %u)\n", db, db ? dev_sum(db, b->size()) : 0u, 4u * 2000u);
  void* dev = nullptr;
  (void) hipMalloc(&dev, 1 << 20);
  SHOW(hipMemcpy(dev, n1->data(), n1->size(), hipMemcpyHostToDevice));
  SHOW(hipMemcpy(dev, n2->data(), n2->size(), hipMemcpyHostToDevice));
  SHOW(hipMemcpy(n2->data(), dev, n2->size(), hipMemcpyDeviceToHost));
  SHOW(hipMemcpy(dev, n3->data(), n3->size(), hipMemcpyHostToDevice));
  // a copy straddling the end of a into n2
  SHOW(hipMemcpy(dev, a->data() + 2900, 300, hipMemcpyHostToDevice));
  SHOW(hipMemcpy(dev, a->data() + 100, 200, hipMemcpyHostToDevice));
  SHOW(hipMemcpyAsync(dev, a->data(), 3000, hipMemcpyHostToDevice, 0));
  SHOW(hipDeviceSynchronize());
  SHOW(hipHostUnregister(a->data()));
  std::printf("  after unregistering a: b device sum %u (want %u)\n", db ? dev_sum(db, b->size()) : 0u, 4u * 2000u);
  SHOW(hipMemcpy(dev, b->data(), b->size(), hipMemcpyHostToDevice));
  SHOW(hipHostUnregister(a->data()));
  SHOW(hipHostUnregister(b->data()));
  SHOW(hipDeviceSynchronize());
  // a large (mmap'd) block: data at page + 16
  std::vector<unsigned char>* big = new std::vector<unsigned char>(1 << 22, 6);
  std::printf("big %p (page offset %lu)\n", (void*) big->data(), (unsigned long) ((uintptr_t) big->data() & 4095));
  SHOW(hipHostRegister(big->data(), big->size(), hipHostRegisterMapped));
  void* dbig = nullptr;
  SHOW(hipHostGetDevicePointer(&dbig, big->data(), 0));
  SHOW(hipMemcpy(dev, big->data() + 1000, 1 << 19, hipMemcpyHostToDevice));
  SHOW(hipHostUnregister(big->data()));
  SHOW(hipDeviceSynchronize());
  std::printf("probe done\n");
  return 0;
}
