// Probe: are large by-value kernel arguments deep-copied into captured hipGraph kernel
// nodes?  Each case captures k<N>(Big<N>{seed + i}, out), clobbers the host stack, replays
// twice and checks out[i] == seed + i.  The kernel only copies its argument: no pointer in
// the argument is dereferenced, so a stale capture shows up as wrong values, not a fault.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

template <int N> struct Big { int v[N]; };

template <int N>
__global__ void copy_arg(Big<N> b, int *out) {
    for (int i = threadIdx.x; i < N; i += blockDim.x) out[i] = b.v[i];
}

__attribute__((noinline)) void clobber() {
    volatile char junk[65536];
    for (int i = 0; i < 65536; ++i) junk[i] = (char)0xA5;
}

template <int N>
__attribute__((noinline)) hipGraphExec_t capture(hipStream_t s, int *out, int seed) {
    Big<N> b;
    for (int i = 0; i < N; ++i) b.v[i] = seed + i;
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
    copy_arg<N><<<1, 256, 0, s>>>(b, out);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    return ge;
}

template <int N>
int run_case(hipStream_t s) {
    int *out;
    hipMalloc(&out, N * sizeof(int));
    hipGraphExec_t ge = capture<N>(s, out, 1000);
    int bad = 0;
    for (int rep = 0; rep < 2; ++rep) {
        clobber();
        hipMemsetAsync(out, 0, N * sizeof(int), s);
        hipGraphLaunch(ge, s);
        static int host[8192];
        hipMemcpyAsync(host, out, N * sizeof(int), hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        for (int i = 0; i < N; ++i) bad += host[i] != 1000 + i;
    }
    printf("by-value arg %6zu B: %s (%d wrong of %d)\n", sizeof(Big<N>), bad ? "STALE" : "ok", bad, 2 * N);
    hipGraphExecDestroy(ge);
    hipFree(out);
    return bad;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int bad = 0;
    bad += run_case<64>(s);
    bad += run_case<256>(s);
    bad += run_case<512>(s);
    bad += run_case<1000>(s);
    bad += run_case<1100>(s);
    bad += run_case<2000>(s);
    printf("%s\n", bad ? "large kernel arguments are NOT captured by value" : "all captured by value");
    return 0;
}
