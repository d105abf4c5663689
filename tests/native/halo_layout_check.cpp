// Host-side check of the halo slot maps (iblb_device.h, iblb_kernels.h): every halo a slab
// exchanges carries exactly the column-planes its boundary kernels pull, each in one slot, and
// the sender's view of a slot is the inverse of the receiver's.  Built and run by
// tests/test_halo_layout.py on the CPU (no GPU needed: the maps are constexpr host/device code).
#include <cstdio>
#include <set>

#include "iblb_kernels.h"

using namespace iblb;

static int fails = 0;
#define CHECK(c, ...)                                 \
    do {                                              \
        if (!(c)) {                                   \
            std::printf("FAIL %s: ", #c);             \
            std::printf(__VA_ARGS__);                 \
            std::printf("\n");                        \
            ++fails;                                  \
        }                                             \
    } while (0)

int main() {
    for (int K = 3; K <= 6; ++K) {
        const int ns = deep_slots(K);
        for (int side = 0; side < 2; ++side) {
            const bool left = side == 0;  // halo received from the left neighbour
            std::set<int> used;
            int carried = 0;
            for (int d = 0; d < K; ++d)
                for (int k = 0; k < 9; ++k) {
                    const int s = deep_slot(left, d, k, K);
                    if (s < 0) continue;
                    ++carried;
                    CHECK(s < ns, "K=%d d=%d k=%d slot %d >= %d", K, d, k, s, ns);
                    CHECK(used.insert(s).second, "K=%d slot %d used twice", K, s);
                    // the sender's view of this slot (it sends to its right when we receive
                    // from the left)
                    CHECK(deep_send_depth(s, K) == d, "K=%d s=%d depth %d != %d", K, s, deep_send_depth(s, K), d);
                    CHECK(deep_send_plane(left, s, K) == k, "K=%d s=%d plane %d != %d", K, s,
                          deep_send_plane(left, s, K), k);
                }
            CHECK(carried == ns, "K=%d carried %d != %d", K, carried, ns);
            // slots 0-2 are the one-step halo (a one-step launch can follow a deep exchange)
            for (int p = 0; p < 3; ++p) {
                const int k = left ? left_plane(p) : right_plane(p);
                CHECK(deep_slot(left, 0, k, K) == halo_slot(k), "K=%d one-step plane %d", K, k);
            }
            // K = 3 is the IB halo
            if (K == 3)
                for (int d = 0; d < 3; ++d)
                    for (int k = 0; k < 9; ++k)
                        CHECK(deep_slot(left, d, k, 3) == ib_slot(left, d, k), "K=3 d=%d k=%d vs ib_slot", d, k);
            // every column-plane the boundary sweep pulls beyond the edge is carried: level-1
            // columns reach K-1 beyond the edge, their pulls one more; walls use the column's own
            // planes 5, 6 (top) and 7, 8 (bottom)
            for (int x1 = 1; x1 <= K - 1; ++x1) {   // level-1 column x1 beyond the edge
                for (int k = 0; k < 9; ++k) {
                    const int c = left ? cx(k) : -cx(k);   // columns further out for the pull
                    const int d = x1 - 1 + c;              // depth of the pulled column
                    if (d < 0) continue;                   // inside the slab
                    CHECK(deep_slot(left, d, k, K) >= 0, "K=%d pull col %d plane %d not carried", K, d, k);
                }
                for (int k : {5, 6, 7, 8})
                    CHECK(deep_slot(left, x1 - 1, k, K) >= 0, "K=%d wall plane %d of col %d not carried", K, k, x1 - 1);
            }
        }
    }
    // the 2-step halo: slots 0-2 the one-step halo, sender / receiver consistent
    for (int s = 0; s < 9; ++s) {
        for (int side = 0; side < 2; ++side) {
            const bool to_left = side == 0;
            const int k = sweep_send_plane(to_left, s);
            const int d = s < 6 ? 0 : 1;
            CHECK(sweep_slot(!to_left, d, k) == s, "2-step slot %d (to_left %d) plane %d", s, to_left, k);
        }
    }
    std::printf(fails ? "halo layout: %d failures\n" : "halo layout: ok\n", fails);
    return fails ? 1 : 0;
}
