// Standalone repro (measurement / diagnosis only, not part of the library;
// VERDICT r5 "what's weak" #1): does a memset node of a hipGraph write what
// it was captured with on every replay?
//
// Round 5 saw the adaptive-mask thresholds of a replayed one-call graph read
// back as 0 / -7.4e8 from its second replay on, with a captured
// hipMemsetAsync(hist, 0, ...) clearing the histogram buffer first.  -7.4e8 is
// dynamic_range = hmax - 1024 with hmax = 0xD3D3D3D3 (-741093421): every byte
// of the max word was 0xD3 -- a byte fill with the wrong value, not a stray
// pointer store.  torch.cuda.graph (keep_graph=False) destroys the captured
// hipGraph_t right after hipGraphInstantiate, so this program checks whether
// the instantiated memset node still depends on the destroyed graph's memory.
//
// Each graph: k_dirty (fills H with 0xffffffff) -> clear(H) -> k_check (counts
// the non-zero words of H, keeps the first).  Between replays the host heap is
// churned: blocks of 8..512 B allocated, filled with the marker byte 0xA5,
// freed.  Variants:
//   memset_keep        hipMemsetAsync captured, the graph kept alive
//   memset_destroy     hipMemsetAsync captured, graph destroyed after instantiate
//                      (torch.cuda.graph's lifecycle)
//   memset_d32_destroy hipMemsetD32Async captured, graph destroyed
//   memset_node_destroy  the graph built with hipGraphAddMemsetNode, destroyed
//   zero_kernel_destroy  a zeroing kernel instead of the memset (the library's
//                      k_zero since round 5), graph destroyed
// One JSON line per replay: non-zero words left after the clear, the first one.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kWords = 2176;  // the library's per-view histogram: 8 replicas x 272 words (8704 B)

__global__ void k_dirty(unsigned* h, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) h[i] = 0xffffffffu;
}
__global__ void k_zero(unsigned* h, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) h[i] = 0u;
}
// out[0] = non-zero words, out[1] = the first non-zero word's value, out[2] = its index
__global__ void k_check(const unsigned* h, int n, unsigned* out) {
  __shared__ unsigned cnt, first, idx;
  if (threadIdx.x == 0) {
    cnt = 0u;
    first = 0u;
    idx = 0xffffffffu;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    if (h[i]) {
      atomicAdd(&cnt, 1u);
      atomicMin(&idx, static_cast<unsigned>(i));
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = cnt;
    out[2] = idx;
    out[1] = idx < static_cast<unsigned>(n) ? h[idx] : 0u;
  }
}

static void churn(int round) {
  std::vector<void*> keep;
  for (int i = 0; i < 4000; ++i) {
    const size_t n = 8 + static_cast<size_t>((i * 2654435761u + round) % 505);
    void* p = malloc(n);
    memset(p, 0xA5, n);
    if (i % 3) free(p);
    else keep.push_back(p);
  }
  for (void* p : keep) free(p);
}

int main(int argc, char** argv) {
  const int replays = argc > 1 ? atoi(argv[1]) : 6;
  unsigned *h, *out;
  CHECK(hipMalloc(&h, sizeof(unsigned) * kWords));
  CHECK(hipMalloc(&out, 16));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* names[] = {"memset_keep", "memset_destroy", "memset_d32_destroy", "memset_node_destroy",
                         "zero_kernel_destroy"};
  int bad_total = 0;
  for (int v = 0; v < 5; ++v) {
    const std::string name = names[v];
    hipGraph_t g = nullptr;
    if (name == "memset_node_destroy") {
      CHECK(hipGraphCreate(&g, 0));
      hipGraphNode_t n0, n1, n2;
      hipKernelNodeParams kp{};
      int nw = kWords;
      void* a0[] = {&h, &nw};
      kp.func = reinterpret_cast<void*>(k_dirty);
      kp.gridDim = dim3(1);
      kp.blockDim = dim3(256);
      kp.kernelParams = a0;
      CHECK(hipGraphAddKernelNode(&n0, g, nullptr, 0, &kp));
      hipMemsetParams mp{};
      mp.dst = h;
      mp.value = 0;
      mp.elementSize = 1;
      mp.width = sizeof(unsigned) * kWords;
      mp.height = 1;
      mp.pitch = 0;
      CHECK(hipGraphAddMemsetNode(&n1, g, &n0, 1, &mp));
      void* a2[] = {&h, &nw, &out};
      kp.func = reinterpret_cast<void*>(k_check);
      kp.kernelParams = a2;
      CHECK(hipGraphAddKernelNode(&n2, g, &n1, 1, &kp));
    } else {
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      hipLaunchKernelGGL(k_dirty, dim3(1), dim3(256), 0, s, h, kWords);
      if (name == "zero_kernel_destroy") hipLaunchKernelGGL(k_zero, dim3(1), dim3(256), 0, s, h, kWords);
      else if (name == "memset_d32_destroy") CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h), 0, kWords, s));
      else CHECK(hipMemsetAsync(h, 0, sizeof(unsigned) * kWords, s));
      hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, s, h, kWords, out);
      CHECK(hipStreamEndCapture(s, &g));
    }
    hipGraphExec_t ge;
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    if (name != "memset_keep") CHECK(hipGraphDestroy(g));
    for (int r = 0; r < replays; ++r) {
      churn(r + 17 * v);
      CHECK(hipMemset(out, 0x77, 16));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipStreamSynchronize(s));
      unsigned o[4];
      CHECK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
      const bool bad = o[0] != 0u;
      bad_total += bad;
      printf("{\"variant\": \"%s\", \"replay\": %d, \"nonzero_words\": %u, \"first_word\": \"0x%08x\", "
             "\"first_index\": %d, \"ok\": %s}\n",
             name.c_str(), r, o[0], o[1], static_cast<int>(o[2]), bad ? "false" : "true");
      fflush(stdout);
    }
    CHECK(hipGraphExecDestroy(ge));
    if (name == "memset_keep") CHECK(hipGraphDestroy(g));
  }
  int rt = 0;
  (void)hipRuntimeGetVersion(&rt);
  printf("{\"hip_runtime_version\": %d, \"bad_replays\": %d}\n", rt, bad_total);
  return 0;
}
