// Cost-balanced stream-K ranges of the attention kernel (rf_attn_schedule): host code only, split out of
// attention.hip so that it builds and runs under AddressSanitizer / UBSan on a machine without a GPU
// (make asan: tests/host/host_asan.cpp, tests/test_host_asan.py).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "common.h"

namespace {
constexpr int KT = rf::ATTN_KT;             // keys per tile (attention.hip)
constexpr int QB5 = rf::ATTN_QB;            // query rows per stream-K unit
constexpr int SK5_MAX_GRID = rf::ATTN_MAX_GRID;
}  // namespace

// ---------------------------------------------------------------------------------------------
// Cost-balanced stream-K ranges (rf_attn_schedule).  With equal tile counts per workgroup the launch
// ends with the owners of units cut three ways: a workgroup whose range lies inside one unit ("mid")
// has one piece (one prologue, one publish) and finishes ~14 % early, while the owner of that unit
// has two pieces and merges two partials (bench shape, per-role lifetimes from the s_memtime stamps of
// tools/attn_ablate.py stamps: mid 222k, owners of 3-way units 257k, others 246k cycles).  Here every
// piece costs a prologue, its tiles, and a publish (non-first piece of its unit) or a finish (first
// piece: one merge per later piece, each after that piece's publish, then the O store), and the
// ranges are chosen backwards from the last workgroup (whose successors' publish times are then known)
// so that every workgroup finishes by a common time T, the smallest T that covers all tiles.
namespace {
struct SkCost {
    // shader cycles, refit in round 5 on the kernel whose next piece's loads go out ahead of the previous piece's
    // stores (prologues 17.6k -> 7.2k per two-piece workgroup; profiles/r5b_attn_prefetch_ab.txt): the A/B of
    // tools/gpu.sh costab measured 130.8 us per stage-1 launch against 131.3 us on the round-4 constants
    // (3170, 8700, 8500, 9800, 6000) and 131.7 us on (3080, 6000, 6500, 8800, 3000) (profiles/r5c_attn_cost_ab.txt)
    double tile = 3080, pro = 5000, pub = 5000, merge = 8800, store = 2500;
};

struct SkUnits {
    std::vector<int64_t> base;  // first tile of problem i
    std::vector<int64_t> nt;    // tiles per unit of problem i (0: problem holds no tiles)
    int64_t total = 0;
    void unit_of(int64_t x, int64_t& us, int64_t& ue) const {  // [start, end) of the unit holding tile x
        int64_t i = (int64_t)(std::upper_bound(base.begin(), base.end(), x) - base.begin()) - 1;
        while (nt[i] == 0) --i;
        const int64_t u = (x - base[i]) / nt[i];
        us = base[i] + u * nt[i];
        ue = us + nt[i];
    }
};

// finish time of workgroup w with range [a, b), given the later workgroups' bounds and publish times;
// *pub = the publish time of its first piece when that piece is a unit's later piece
double sk_simulate(const SkUnits& U, const SkCost& c, int w, int64_t a, int64_t b, const std::vector<int64_t>& bnd,
                   const std::vector<double>& pubt, int grid, double* pub) {
    double t = 0;
    *pub = 0;
    for (int64_t x = a; x < b;) {
        int64_t us, ue;
        U.unit_of(x, us, ue);
        const int64_t e = std::min(b, ue);
        t += c.pro + (double)(e - x) * c.tile;
        if (x > us) {
            t += c.pub;
            *pub = t;
        } else {
            if (e < ue) {  // merges in the kernel's order: the last later workgroup first
                int last = w + 1;
                while (last < grid && bnd[last] < ue) ++last;
                for (int cw = last - 1; cw > w; --cw)
                    if (bnd[cw + 1] > bnd[cw]) t = std::max(t, pubt[cw]) + c.merge;
            }
            t += c.store;
        }
        x = e;
    }
    return t;
}

// backward fill with finish time T; returns bnd[0] (0 = every tile placed).  A range is feasible when the
// workgroup finishes by T and its published piece (if any) lands early enough for the owner to merge it
// and store by T; the largest feasible range is found by bisection on its start (the finish time grows
// with the range except at unit boundaries, where a piece changes role).
int64_t sk_fill(const SkUnits& U, const SkCost& c, int grid, double T, std::vector<int64_t>& bnd,
                std::vector<double>& pubt) {
    bnd.assign(grid + 1, 0);
    pubt.assign(grid + 1, 0);
    bnd[grid] = U.total;
    // a published piece must land in time for the owner's merges from it on and its store: a unit's middle piece
    // (the range lies strictly inside one unit) is merged last, so one merge follows; a tail piece is merged
    // first, so one merge follows when the rest of its unit fits one earlier range (a two-way cut, e.g. every
    // cross-attention unit) and two when it needs two (a three-way cut)
    const double avg = (double)U.total / grid;
    auto ok = [&](int w, int64_t a, int64_t b, double* pub) {
        if (sk_simulate(U, c, w, a, b, bnd, pubt, grid, pub) > T) return false;
        int64_t us, ue;
        U.unit_of(a, us, ue);
        const bool mid = a > us && b < ue;
        const int after = (mid || (double)(a - us) <= 1.3 * avg) ? 1 : 2;
        return *pub <= T - after * c.merge - c.store;
    };
    for (int w = grid - 1; w >= 0; --w) {
        const int64_t b = bnd[w + 1];
        double pub = 0;
        // no range holds more than T / tile tiles: search starts in [b - that - 1, b) only
        const int64_t reach = (int64_t)(T / c.tile) + 1;
        int64_t lo = b, hi = 0;  // lo: feasible start (empty range), search [hi, lo)
        if (b > 0 && b <= reach && ok(w, 0, b, &pub)) {
            lo = 0;
        } else if (b > 0) {
            hi = std::max<int64_t>(1, b - reach);
            while (hi < lo) {  // smallest feasible a in [hi, lo]
                const int64_t mid = (hi + lo) / 2;
                if (ok(w, mid, b, &pub)) lo = mid;
                else hi = mid + 1;
            }
            // feasibility is not monotone where the first piece changes role: a start just inside a unit makes a
            // published piece, the unit's first tile an owned one; prefer the owned start when it also fits
            if (lo < b) {
                int64_t us, ue;
                U.unit_of(lo, us, ue);
                if (us < lo && ok(w, us, b, &pub)) lo = us;
            }
        }
        bnd[w] = lo;
        ok(w, lo, b, &pub);
        pubt[w] = lo < b ? pub : 0;
    }
    return bnd[0];
}
// the model's finish time of a given table (every workgroup, successors first so publish times are known)
double sk_span(const SkUnits& U, const SkCost& c, int grid, const std::vector<int64_t>& bnd) {
    std::vector<double> pubt(grid + 1, 0.0);
    double span = 0;
    for (int w = grid - 1; w >= 0; --w) {
        double pub = 0;
        const double t = bnd[w + 1] > bnd[w] ? sk_simulate(U, c, w, bnd[w], bnd[w + 1], bnd, pubt, grid, &pub) : 0.0;
        pubt[w] = pub;
        span = std::max(span, t);
    }
    return span;
}
}  // namespace


namespace {
// One XCD group's ranges (sk_fill + bisection on the common finish time; equal tile counts kept when the model
// prices them no worse), bounds relative to the group's first tile: out[0..grid].
void sk_schedule_group(const SkUnits& U, const SkCost& c, int grid, int64_t* out) {
    if (U.total <= grid) {
        // fewer tiles than workgroups: one whole unit per workgroup, nothing cut, so a unit's result does not
        // depend on the rest of the launch (a view rendered alone equals the same view in a batch)
        int w = 0;
        for (size_t i = 0; i < U.base.size(); ++i)
            if (U.nt[i])
                for (int64_t x = U.base[i]; x < (i + 1 < U.base.size() ? U.base[i + 1] : U.total); x += U.nt[i])
                    out[w++] = x;
        for (; w <= grid; ++w) out[w] = U.total;
        return;
    }
    std::vector<int64_t> bnd;
    std::vector<double> pubt;
    // lo is infeasible (less than the average tile work); hi doubled until feasible
    double lo = (double)U.total * c.tile / grid;
    double hi = 2 * lo + 4 * (c.pro + c.pub + c.merge + c.store);
    while (sk_fill(U, c, grid, hi, bnd, pubt) != 0) {
        lo = hi;
        hi *= 2;
    }
    for (int iter = 0; iter < 60 && hi - lo > 0.25 * c.tile; ++iter) {
        const double mid = 0.5 * (lo + hi);
        (sk_fill(U, c, grid, mid, bnd, pubt) == 0 ? hi : lo) = mid;
    }
    sk_fill(U, c, grid, hi, bnd, pubt);
    std::vector<int64_t> eq(grid + 1);
    for (int w = 0; w <= grid; ++w) eq[w] = U.total * w / grid;
    const std::vector<int64_t>& best = sk_span(U, c, grid, eq) <= sk_span(U, c, grid, bnd) ? eq : bnd;
    for (int w = 0; w <= grid; ++w) out[w] = best[w];
}
}  // namespace

// Cost-balanced stream-K ranges in the forward-progress layout (common.h SkLayout): the units (head x q-block
// of each problem with keys, in problem order) are cut into one contiguous chunk per XCD group, balanced by
// tiles, so a unit never spans two groups (its pieces' blocks share an XCD's L2 when there are 8 groups, and
// an owner only waits on lower-numbered blocks); each chunk is scheduled over its group's blocks by the cost
// model above.  bounds[L] is the first tile of LOGICAL block L (bounds[grid] = total), as the kernel reads it.
extern "C" int rf_attn_schedule(const int32_t* problems, int n_problems, int n_heads, int grid, int64_t* bounds) {
    RF_REQUIRE(problems && bounds && n_problems > 0 && n_heads > 0, "rf_attn_schedule: bad arguments");
    RF_REQUIRE(grid >= 1 && grid <= SK5_MAX_GRID, "rf_attn_schedule: grid %d out of range", grid);
    // every unit as (first tile, tiles): the problems' units in order
    std::vector<int64_t> ustart, unt;
    int64_t total = 0;
    for (int i = 0; i < n_problems; ++i) {
        const int32_t* d = problems + 5 * i;
        RF_REQUIRE(d[1] >= 0 && d[3] >= 0, "rf_attn_schedule: negative length in problem %d", i);
        const int64_t nt = (d[3] + KT - 1) / KT;
        const int64_t nu = nt > 0 ? (int64_t)n_heads * ((d[1] + QB5 - 1) / QB5) : 0;
        for (int64_t u = 0; u < nu; ++u) {
            ustart.push_back(total);
            unt.push_back(nt);
            total += nt;
        }
    }
    const int64_t NU = (int64_t)ustart.size();
    if (total == 0) {
        for (int w = 0; w <= grid; ++w) bounds[w] = 0;
        return RF_OK;
    }
    SkCost c;
    if (const char* env = getenv("RF_ATTN_COST"))  // tile,pro,pub,merge,store (tuning)
        sscanf(env, "%lf,%lf,%lf,%lf,%lf", &c.tile, &c.pro, &c.pub, &c.merge, &c.store);
    const SkLayout lay(grid, NU);
    int64_t u0 = 0;
    for (int g = 0; g < lay.G; ++g) {
        // this group's units: up to the unit boundary nearest its share of the tiles (>= 1 unit per group)
        int64_t u1 = NU;
        if (g + 1 < lay.G) {
            const int64_t target = total * lay.base(g + 1) / grid;
            u1 = (int64_t)(std::lower_bound(ustart.begin(), ustart.end(), target) - ustart.begin());
            if (u1 > 0 && u1 < NU && target - ustart[u1 - 1] < ustart[u1] - target) --u1;  // nearer boundary
            u1 = std::max(u1, u0 + 1);
            u1 = std::min(u1, NU - (lay.G - g - 1));
        }
        SkUnits U;  // the chunk as runs of equal-size units, relative tiles
        const int64_t t0 = ustart[u0];
        for (int64_t u = u0; u < u1; ++u) {
            if (u == u0 || unt[u] != unt[u - 1] || U.nt.back() == 0) {
                U.base.push_back(ustart[u] - t0);
                U.nt.push_back(unt[u]);
            }
            U.total += unt[u];
        }
        const int nb = lay.size(g), b0 = lay.base(g);
        std::vector<int64_t> rel(nb + 1);
        sk_schedule_group(U, c, nb, rel.data());
        for (int i = 0; i < nb; ++i) bounds[b0 + i] = t0 + rel[i];
        u0 = u1;
    }
    bounds[grid] = total;
    return RF_OK;
}

