// HIP-only reduction of the two-lane GraphedRAFT capture: does hipStreamEndCapture
// crash on the stream topology alone, without torch's allocator, events or kernels?
//
// The topology mirrors one test-mode RAFT forward with pair lanes (methods/raft/model/raft.py:_forward and
// _split_update_lanes, model/update.py SplitUpdate.update), with empty kernels writing one float each:
//   C  = the capture stream (graph.py's warm-up stream)
//   E0 = C's side stream slot 0 (cnet encoder; ALSO lane 0's flow-branch side stream: both are _side_stream(dev, 0)
//        with owner C), E1 = C's slot 1 (fnet's second image)
//   L1 = lane 1 (slot 101 of C), S1 = L1's side stream (slot 201 with owner L1)
// Every fork / join is torch's wait_stream: a fresh event (hipEventDisableTiming) recorded on the producer, waited on
// by the consumer, destroyed right after the wait (the temporary Event's refcount drops at once in Python).
//
// modes (argv[1]):
//   nolaneside -- lanes without their side streams (what graph.py captures today: known to work)
//   lane1side  -- lane 1's side stream only (a fork from a stream that itself joined the capture by a fork)
//   lane0side  -- lane 0's side stream only (E0 re-forked from C after the encoders joined it)
//   full       -- both (the configuration that segfaults in capture_end under torch)
//   keepevents -- full, but every event kept alive until after hipStreamEndCapture
// argv[2]: iterations (12), argv[3]: kernels per modelled op (1), argv[4]: 1 = hipSetDevice(0) before every launch,
// record and wait (torch's device guards make ~1.8 such calls per operation during a capture: r6s6's log).
// Prints one line per phase; the final line "RESULT <mode> ok replay_equal=<0|1>" or an error status.
// Build: hipcc --offload-arch=gfx950 -O2 -o build/exp/capture_fork_repro tools/exp/capture_fork_repro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                          \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) {                                                                            \
      std::printf("HIP error %d (%s) at %s:%d: %s\n", (int)e_, hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      std::fflush(stdout);                                                                             \
      std::exit(3);                                                                                    \
    }                                                                                                  \
  } while (0)

__global__ void tick(float* p, int slot) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[slot] = p[slot] * 0.5f + (float)slot;
}

namespace {

bool g_keep = false;
int g_per = 1;  // kernels per modelled op (torch's in-place mul_ + add_ = 2)
bool g_setdev = false;  // hipSetDevice(0) before every launch / record / wait, as torch's device guards do
std::vector<hipEvent_t> g_kept;
float* g_buf = nullptr;
int g_slot = 0;

// torch.cuda.Stream.wait_stream(other): consumer waits for everything enqueued on producer so far
void wait_stream(hipStream_t consumer, hipStream_t producer) {
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  if (g_setdev) CK(hipSetDevice(0));
  CK(hipEventRecord(ev, producer));
  if (g_setdev) CK(hipSetDevice(0));
  CK(hipStreamWaitEvent(consumer, ev, 0));
  if (g_keep)
    g_kept.push_back(ev);
  else
    CK(hipEventDestroy(ev));
}

void k(hipStream_t s, int n = 1) {
  for (int i = 0; i < n * g_per; ++i) {
    if (g_setdev) CK(hipSetDevice(0));
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, g_buf, g_slot % 4096);
    ++g_slot;
  }
  CK(hipGetLastError());
}

// one forward: encoders on C / E0 / E1, then `iters` lane iterations (lane 0 on C, lane 1 on L1)
void forward(hipStream_t C, hipStream_t E0, hipStream_t E1, hipStream_t L1, hipStream_t S1, bool side0, bool side1,
             int iters) {
  g_slot = 0;
  k(C, 2);                 // normalize, pad
  wait_stream(E1, C);      // fnet image 1 on E1
  k(E1, 12);
  k(C, 3);                 // stem patches
  wait_stream(E0, C);      // cnet on E0
  k(E0, 12);
  k(C, 12);                // fnet image 0
  wait_stream(C, E1);
  k(C, 1);                 // pyramid
  wait_stream(C, E0);
  k(C, 2);                 // coords
  k(C, 3);                 // lane 0's packs + context terms (side_owner C)
  wait_stream(L1, C);      // lanes fork
  k(L1, 3);                // lane 1's packs + context terms
  for (int it = 0; it < iters; ++it) {
    const bool last = it == iters - 1;
    if (last) wait_stream(L1, C);  // the mask block (need)
    // lane 0 on C
    if (side0) {
      wait_stream(E0, C);
      k(E0, 3);            // flow prep, convf1, convf2
      k(C, 2);             // convc1 (fused lookup), convc2
      wait_stream(C, E0);
    } else {
      k(C, 5);
    }
    k(C, 8);               // motion conv, GRU x4, flow head x2 (+ mask head on the last)
    // lane 1 on L1
    if (side1) {
      wait_stream(S1, L1);
      k(S1, 3);
      k(L1, 2);
      wait_stream(L1, S1);
    } else {
      k(L1, 5);
    }
    k(L1, 8);
    if (last) {
      wait_stream(C, L1);
      k(C, 1);             // convex upsampling
    }
  }
  wait_stream(C, L1);
  k(C, 1);                 // coords1 - coords0
}

}  // namespace

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "full";
  bool side0 = true, side1 = true;
  if (!std::strcmp(mode, "nolaneside")) {
    side0 = side1 = false;
  } else if (!std::strcmp(mode, "lane1side")) {
    side0 = false;
  } else if (!std::strcmp(mode, "lane0side")) {
    side1 = false;
  } else if (!std::strcmp(mode, "keepevents")) {
    g_keep = true;
  } else if (std::strcmp(mode, "full") != 0) {
    std::printf("unknown mode %s\n", mode);
    return 2;
  }
  const int iters = argc > 2 ? std::atoi(argv[2]) : 12;
  if (argc > 3) g_per = std::atoi(argv[3]);
  if (argc > 4) g_setdev = std::atoi(argv[4]) != 0;
  CK(hipSetDevice(0));
  CK(hipMalloc(&g_buf, 4096 * sizeof(float)));
  hipStream_t C, E0, E1, L1, S1;
  for (hipStream_t* s : {&C, &E0, &E1, &L1, &S1}) CK(hipStreamCreateWithFlags(s, hipStreamNonBlocking));

  // eager reference
  CK(hipMemsetAsync(g_buf, 0, 4096 * sizeof(float), C));
  forward(C, E0, E1, L1, S1, side0, side1, iters);
  CK(hipStreamSynchronize(C));
  std::vector<float> ref(4096), got(4096);
  CK(hipMemcpy(ref.data(), g_buf, 4096 * sizeof(float), hipMemcpyDeviceToHost));
  std::printf("eager ok (%d launches)\n", g_slot);
  std::fflush(stdout);

  // capture (global mode, as torch.cuda.graph's default capture_error_mode)
  CK(hipMemsetAsync(g_buf, 0, 4096 * sizeof(float), C));
  CK(hipStreamSynchronize(C));
  hipGraph_t graph = nullptr;
  CK(hipStreamBeginCapture(C, hipStreamCaptureModeGlobal));
  forward(C, E0, E1, L1, S1, side0, side1, iters);
  std::printf("captured %d launches; calling hipStreamEndCapture\n", g_slot);
  std::fflush(stdout);
  CK(hipStreamEndCapture(C, &graph));
  std::printf("end capture ok\n");
  std::fflush(stdout);
  for (hipEvent_t ev : g_kept) CK(hipEventDestroy(ev));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(exec, C));
  CK(hipStreamSynchronize(C));
  CK(hipMemcpy(got.data(), g_buf, 4096 * sizeof(float), hipMemcpyDeviceToHost));
  const bool eq = std::memcmp(got.data(), ref.data(), 4096 * sizeof(float)) == 0;
  std::printf("RESULT %s ok nodes=%zu replay_equal=%d\n", mode, nodes, eq ? 1 : 0);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  for (hipStream_t s : {C, E0, E1, L1, S1}) CK(hipStreamDestroy(s));
  CK(hipFree(g_buf));
  return eq ? 0 : 1;
}
