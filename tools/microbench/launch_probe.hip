// Host cost of enqueuing one batch's launch sequence: K kernel launches on a stream one by one
// against one hipGraphLaunch of the same K kernel nodes (captured once), and against updating the
// graph's kernel arguments before each launch (hipGraphExecKernelNodeSetParams on every node).
// Kernels are trivial (one workgroup, one store), so the numbers are the host's enqueue cost and
// the GPU's per-dispatch cost, not compute.
//   hipcc --offload-arch=gfx950 -O2 launch_probe.hip -o launch_probe && ./launch_probe [K] [reps]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Args {
  unsigned* out;
  unsigned a, b, c, d;
  const void* p0;
  const void* p1;
  const void* p2;
};

__global__ void k_touch(Args A) {
  if (threadIdx.x == 0) A.out[blockIdx.x] = A.a + A.b + A.c + A.d;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 17;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  unsigned* d;
  CK(hipMalloc(&d, 4096));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Args A{d, 1, 2, 3, 4, d, d, d};
  // warm up the code object
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, A);
  CK(hipStreamSynchronize(st));

  // (1) K plain launches per "batch"
  std::vector<double> t_plain;
  for (int r = 0; r < reps; ++r) {
    double t0 = now_us();
    for (int k = 0; k < K; ++k) {
      A.a = r + k;
      hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, A);
    }
    t_plain.push_back(now_us() - t0);
    if (r % 8 == 7) CK(hipStreamSynchronize(st));
  }
  CK(hipStreamSynchronize(st));
  double t0 = now_us();
  for (int r = 0; r < reps; ++r)
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, A);
  CK(hipStreamSynchronize(st));
  const double gpu_plain = (now_us() - t0) / reps;

  // (2) the same K kernels captured into one graph
  hipGraph_t g;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, A);
  CK(hipStreamEndCapture(st, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CK(hipGraphGetNodes(g, nodes.data(), &nn));
  for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  std::vector<double> t_graph;
  for (int r = 0; r < reps; ++r) {
    double t1 = now_us();
    CK(hipGraphLaunch(ge, st));
    t_graph.push_back(now_us() - t1);
    if (r % 8 == 7) CK(hipStreamSynchronize(st));
  }
  CK(hipStreamSynchronize(st));
  t0 = now_us();
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  const double gpu_graph = (now_us() - t0) / reps;

  // (3) new kernel arguments on every node, then one launch
  std::vector<double> t_upd;
  for (int r = 0; r < reps; ++r) {
    double t1 = now_us();
    for (size_t i = 0; i < nn; ++i) {
      hipKernelNodeParams p;
      CK(hipGraphKernelNodeGetParams(nodes[i], &p));
      Args B = A;
      B.a = r + (unsigned)i;
      void* kp[] = {&B};
      p.kernelParams = kp;
      CK(hipGraphExecKernelNodeSetParams(ge, nodes[i], &p));
    }
    CK(hipGraphLaunch(ge, st));
    t_upd.push_back(now_us() - t1);
    CK(hipStreamSynchronize(st));
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("{\"kernels\": %d, \"reps\": %d, \"plain_host_us\": %.1f, \"plain_gpu_us\": %.1f, "
         "\"graph_host_us\": %.1f, \"graph_gpu_us\": %.1f, \"graph_setparams_host_us\": %.1f}\n",
         K, reps, med(t_plain), gpu_plain, med(t_graph), gpu_graph, med(t_upd));
  return 0;
}
