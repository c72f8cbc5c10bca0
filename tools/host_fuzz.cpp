// host_fuzz.cpp -- sanitizer harness for the composite plan (plan_core.h: the host plan behind
// pano_plan_composite and the device plan kernel plan_device run the same code).  Built with
// -fsanitize=address,undefined by tools/host_sanitize.sh and run on random and adversarial
// shift / pair arrays: NaN, infinities, huge offsets, sign flips, 1..kMaxN frames.  Checks that
// every call returns a status and that PANO_OK plans are self-consistent (every step's canvas
// and frame lie inside the final canvas).  Prints one JSON line; exit status 0 iff clean.
//
//   host_fuzz [iterations] [seed]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../vfx_image_stitching_amd/csrc/plan_core.h"

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t next_u64() {   // splitmix64
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
double uni() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }

double wild(double typical) {
    switch (next_u64() % 16) {
    case 0: return NAN;
    case 1: return INFINITY;
    case 2: return -INFINITY;
    case 3: return 1e300 * (uni() - 0.5);
    case 4: return 4e9 * (uni() - 0.5);
    case 5: return 0.0;
    default: return typical * (2 * uni() - 1);
    }
}

constexpr int kMaxN = 400;

}  // namespace

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    if (argc > 2) g_state = strtoull(argv[2], nullptr, 10);
    long ok = 0, refused = 0, bad = 0, fast_diff = 0;
    std::vector<double> shifts, pairs;
    std::vector<pano_step> steps;
    std::vector<int32_t> tmp;
    for (long it = 0; it < iters; ++it) {
        const int n = 1 + (int)(next_u64() % (it % 50 == 0 ? kMaxN : 24));
        const int h = 1 + (int)(next_u64() % 1200), w = 1 + (int)(next_u64() % 2000);
        const bool adversarial = next_u64() % 4 == 0;
        shifts.assign(2 * (size_t)n, 0.0);
        pairs.assign(4 * (size_t)n, 0.0);
        for (int k = 0; k + 1 < n; ++k) {
            // realistic: dx ~ -w/2 .. -w, dy small, the match inside the frames
            const double dx = -(0.3 + 0.7 * uni()) * w, dy = 8 * (uni() - 0.5);
            shifts[2 * k] = adversarial ? wild(3.0 * w) : (next_u64() % 8 ? dx : -dx);
            shifts[2 * k + 1] = adversarial ? wild(h) : dy;
            for (int q = 0; q < 4; ++q) pairs[4 * k + q] = adversarial ? wild(2.0 * w) : uni() * (q % 2 ? h : w);
        }
        steps.assign((size_t)n, pano_step{});
        tmp.assign(5 * (size_t)n, 0);
        int32_t first[2] = {0, 0}, hw[2] = {0, 0};
        const int rc = plan_core([&](int k, double *d) { d[0] = shifts[2 * k]; d[1] = shifts[2 * k + 1]; },
                                 [&](int k, double *d) { for (int q = 0; q < 4; ++q) d[q] = pairs[4 * k + q]; },
                                 n, h, w, steps.data(), first, hw, tmp.data());
        // plan_device's form (per-step constants + the short chain) must be the same plan
        {
            std::vector<pano_step> steps2((size_t)n, pano_step{});
            std::vector<int32_t> tmp2(5 * (size_t)n, 0);
            int32_t first2[2] = {0, 0}, hw2[2] = {0, 0};
            const int rc2 = plan_fast([&](int k, double *d) { d[0] = shifts[2 * k]; d[1] = shifts[2 * k + 1]; },
                                      [&](int k, double *d) { for (int q = 0; q < 4; ++q) d[q] = pairs[4 * k + q]; },
                                      n, h, w, steps2.data(), first2, hw2, tmp2.data());
            bool same = rc2 == rc;
            if (same && rc == PANO_OK)
                same = memcmp(steps2.data(), steps.data(), sizeof(pano_step) * (size_t)(n - 1 > 0 ? n - 1 : 0)) == 0 &&
                       first2[0] == first[0] && first2[1] == first[1] && hw2[0] == hw[0] && hw2[1] == hw[1];
            if (!same) {
                ++fast_diff;
                if (fast_diff <= 5) fprintf(stderr, "plan_fast differs: iteration %ld n %d rc %d / %d\n", it, n, rc, rc2);
            }
        }
        if (rc != PANO_OK) { ++refused; continue; }
        ++ok;
        // consistency of an accepted plan
        bool good = hw[0] >= h && hw[1] >= w && first[0] >= 0 && first[1] >= 0 && first[0] + w <= hw[1] &&
                    first[1] + h <= hw[0];
        for (int i = 0; good && i + 1 < n; ++i) {
            const pano_step &s = steps[i];
            good = s.canvas_x >= 0 && s.canvas_y >= 0 && s.canvas_x + s.canvas_w <= hw[1] &&
                   s.canvas_y + s.canvas_h <= hw[0] && s.frame_x >= 0 && s.frame_y >= 0 &&
                   s.frame_x + w <= hw[1] && s.frame_y + h <= hw[0];
        }
        if (!good) {
            if (++bad <= 5) fprintf(stderr, "inconsistent plan: iteration %ld n %d h %d w %d\n", it, n, h, w);
        }
    }
    printf("{\"iterations\": %ld, \"ok\": %ld, \"refused\": %ld, \"inconsistent\": %ld, \"plan_fast_differs\": %ld}\n",
           iters, ok, refused, bad, fast_diff);
    return (bad || fast_diff) ? 1 : 0;
}
