// Probe: host time per kernel launch against the size of the kernel-argument
// struct (16 B .. 16 KiB), launched back to back on one stream (an empty
// kernel that reads one word of its arguments), and the same five launches
// replayed as a hipGraph.  Prints microseconds of host time per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

template <int N>
struct Big {
  unsigned v[N];
};
template <int N>
__global__ void k(Big<N> b, unsigned* out) {
  if (threadIdx.x == 0 && b.v[N - 1] == 0xdeadbeefu) out[blockIdx.x] = b.v[0];
}

// a kernel that keeps the GPU busy for about `cycles` clocks
template <int N>
__global__ void busy(Big<N> b, unsigned* out, long long cycles) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && b.v[N - 1] == 0xdeadbeefu) out[blockIdx.x] = b.v[0];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int N>
void run(hipStream_t st, unsigned* d) {
  static Big<N> b;
  for (int i = 0; i < N; ++i) b.v[i] = i;
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k<N>, dim3(64), dim3(256), 0, st, b, d);
  hipStreamSynchronize(st);
  const int R = 2000;
  double best = 1e30;
  for (int rep = 0; rep < 3; ++rep) {
    const double t0 = now_us();
    for (int i = 0; i < R; ++i) {
      b.v[0] = i;
      hipLaunchKernelGGL(k<N>, dim3(64), dim3(256), 0, st, b, d);
    }
    const double t1 = now_us();
    hipStreamSynchronize(st);
    const double t2 = now_us();
    if ((t1 - t0) / R < best) best = (t1 - t0) / R;
    if (rep == 2) printf("kernarg %6zu B: host %.2f us/launch (enqueue), %.2f us/launch incl. drain\n", sizeof(Big<N>), best, (t2 - t0) / R);
  }
}

template <int N>
void run_graph(hipStream_t st, unsigned* d) {
  static Big<N> b;
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int j = 0; j < 5; ++j) hipLaunchKernelGGL(k<N>, dim3(64), dim3(256), 0, st, b, d);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  size_t nn = 0;
  hipGraphGetNodes(g, nullptr, &nn);
  hipGraphNode_t nodes[8];
  hipGraphGetNodes(g, nodes, &nn);
  for (int i = 0; i < 20; ++i) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  const int R = 400;
  const double t0 = now_us();
  for (int i = 0; i < R; ++i) {
    b.v[0] = i;  // new arguments for every node, as a replay with updated jobs would need
    for (size_t j = 0; j < nn; ++j) {
      hipKernelNodeParams p;
      hipGraphKernelNodeGetParams(nodes[j], &p);
      void* args[2] = {&b, &d};
      p.kernelParams = args;
      hipGraphExecKernelNodeSetParams(ge, nodes[j], &p);
    }
    hipGraphLaunch(ge, st);
  }
  const double t1 = now_us();
  hipStreamSynchronize(st);
  const double t2 = now_us();
  printf("graph of 5, kernarg %6zu B, params updated: host %.2f us per 5 launches, %.2f incl. drain\n", sizeof(Big<N>),
         (t1 - t0) / R, (t2 - t0) / R);
  const double t3 = now_us();
  for (int i = 0; i < R; ++i) hipGraphLaunch(ge, st);
  const double t4 = now_us();
  hipStreamSynchronize(st);
  printf("graph of 5, kernarg %6zu B, replay only: host %.2f us per 5 launches\n", sizeof(Big<N>), (t4 - t3) / R);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
}

// five different kernels (template instances) of ~10 us each, back to back
// as a C1 iteration issues them, 40 rounds: host time per launch while the
// GPU is busy
template <int N>
void run_busy(hipStream_t st, unsigned* d) {
  static Big<N + 4> b;  // (the larger instances read a prefix of it)
  const long long cyc = 10 * 100;  // wall_clock64 runs at 100 MHz: 10 us
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(busy<N>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N>*>(&b), d, cyc);
  hipStreamSynchronize(st);
  const int R = 40;
  const double t0 = now_us();
  for (int i = 0; i < R; ++i) {
    hipLaunchKernelGGL(busy<N>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N>*>(&b), d, cyc);
    hipLaunchKernelGGL(busy<N + 1>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N + 1>*>(&b), d, cyc);
    hipLaunchKernelGGL(busy<N + 2>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N + 2>*>(&b), d, cyc);
    hipLaunchKernelGGL(busy<N + 3>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N + 3>*>(&b), d, cyc);
    hipLaunchKernelGGL(busy<N + 4>, dim3(256), dim3(256), 0, st, *reinterpret_cast<Big<N + 4>*>(&b), d, cyc);
  }
  const double t1 = now_us();
  hipStreamSynchronize(st);
  const double t2 = now_us();
  printf("busy GPU, 5 kernels x %d rounds, kernarg %zu B: host %.2f us/launch (enqueue), GPU %.2f us/launch\n", R,
         sizeof(Big<N>), (t1 - t0) / (5 * R), (t2 - t0) / (5 * R));
}

int main() {
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  unsigned* d;
  hipMalloc(&d, 64 * 4);
  run<4>(st, d);
  run<64>(st, d);
  run<256>(st, d);
  run<1024>(st, d);
  run<2048>(st, d);
  run<4096>(st, d);
  run_busy<4>(st, d);
  run_busy<1024>(st, d);
  run_graph<4>(st, d);
  run_graph<1024>(st, d);
  hipFree(d);
  return 0;
}
