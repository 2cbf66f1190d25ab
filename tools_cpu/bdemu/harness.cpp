// tools_cpu/bdemu harness: one dm_sort_nondominated call of the emulated
// library on a population read from a case file, checked front by front
// against a brute-force non-dominated sort (deap/tools/emo.py:53-117: u
// dominates v iff u >= v in every weighted objective and > in one), and
// against the reference's own order when the case file carries it (the
// golden vectors of tests/golden/nsga2.npz, written by make_cases.py).
//
// Case file (little endian): "BDE1", int64 n, int32 m, int64 k,
// double wvalues[n m], int64 nexp, int32 order[nexp], int32 nfr,
// int32 fstart[nfr + 1] (nexp = 0: no reference order).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "common.hpp"

extern "C" int dm_sort_nondominated(dm_ctx* ctx, const dm_pop* pop, int64_t k,
                                    int32_t first_front_only, int32_t* order,
                                    int32_t* front_start, int32_t* rank, int64_t* nsorted,
                                    int32_t* nfronts);

template <class T>
static T rd(FILE* f) {
    T v;
    if (fread(&v, sizeof(T), 1, f) != 1) {
        fprintf(stderr, "harness: short case file\n");
        exit(2);
    }
    return v;
}

static std::vector<std::vector<int>> brute_fronts(const std::vector<double>& wv, int64_t n, int m,
                                                  int64_t k) {
    auto dom = [&](int64_t a, int64_t b) {
        bool gt = false;
        for (int i = 0; i < m; ++i) {
            const double x = wv[a * m + i], y = wv[b * m + i];
            if (x < y) return false;
            if (x > y) gt = true;
        }
        return gt;
    };
    std::vector<int> cnt(n, 0);
    std::vector<std::vector<int>> by(n);
    for (int64_t a = 0; a < n; ++a)
        for (int64_t b = 0; b < n; ++b)
            if (a != b && dom(a, b)) {
                ++cnt[b];
                by[a].push_back((int)b);
            }
    std::vector<std::vector<int>> fronts;
    std::vector<int> cur;
    for (int64_t v = 0; v < n; ++v)
        if (!cnt[v]) cur.push_back((int)v);
    int64_t done = 0;
    const int64_t N = std::min(n, k);
    while (!cur.empty()) {
        fronts.push_back(cur);
        done += (int64_t)cur.size();
        if (done >= N) break;
        std::vector<int> nxt;
        for (int a : cur)
            for (int b : by[a])
                if (--cnt[b] == 0) nxt.push_back(b);
        cur.swap(nxt);
    }
    return fronts;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: harness CASEFILE [first_front_only]\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    char magic[4];
    if (fread(magic, 1, 4, f) != 4 || std::string(magic, 4) != "BDE1") return 2;
    const int64_t n = rd<int64_t>(f);
    const int m = rd<int32_t>(f);
    const int64_t k = rd<int64_t>(f);
    std::vector<double> wv(n * m);
    for (auto& x : wv) x = rd<double>(f);
    const int64_t nexp = rd<int64_t>(f);
    std::vector<int32_t> eorder(nexp);
    for (auto& x : eorder) x = rd<int32_t>(f);
    const int32_t enfr = rd<int32_t>(f);
    std::vector<int32_t> efs(enfr + 1);
    for (auto& x : efs) x = rd<int32_t>(f);
    fclose(f);

    dm_ctx ctx;
#ifdef EMU_PRE
    ctx.knobs.bd_maxm = getenv("EMU_BD_MAXM") ? atoi(getenv("EMU_BD_MAXM")) : 3;
#endif
    // exact-size "device" buffers, so ASan bounds them as the caller sized them
    double* dwv = (double*)malloc(sizeof(double) * n * m);
    std::copy(wv.begin(), wv.end(), dwv);
    uint8_t* valid = (uint8_t*)malloc(n);
    memset(valid, 1, n);
    void* genes = calloc(n, 32);
    dm_pop pop{};
    pop.genes = genes;
    pop.wvalues = dwv;
    pop.valid = valid;
    pop.n = n;
    pop.stride = 32;
    pop.dim = 2;
    pop.gtype = DM_F64;
    pop.nobj = m;
    int32_t* order = (int32_t*)malloc(4 * std::max<int64_t>(n, 1));
    int32_t* fstart = (int32_t*)malloc(4 * (std::max<int64_t>(n, 1) + 1));
    int32_t* rank = (int32_t*)malloc(4 * std::max<int64_t>(n, 1));
    int64_t nsorted = 0;
    int32_t nfronts = 0;
    const int ffo = argc > 2 ? atoi(argv[2]) : 0;
    const int rc = dm_sort_nondominated(&ctx, &pop, k, ffo, order, fstart, rank, &nsorted, &nfronts);
    printf("n %lld m %d k %lld: rc %d, %d fronts, %lld sorted\n", (long long)n, m, (long long)k, rc,
           nfronts, (long long)nsorted);
    if (rc) return 1;
    auto bf = brute_fronts(wv, n, m, k);
    if (ffo) bf.resize(1);
    bool ok = (int)bf.size() == nfronts;
    for (int fi = 0; ok && fi < nfronts; ++fi) {
        std::vector<int> a(order + fstart[fi], order + fstart[fi + 1]);
        std::vector<int> b = bf[fi];
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        if (a != b) {
            printf("front %d differs from brute force (%zu vs %zu members)\n", fi, a.size(), b.size());
            ok = false;
        }
    }
    printf("fronts == brute force: %s\n", ok ? "yes" : "NO");
    bool eok = true;
    if (nexp && !ffo) {
        eok = nexp == nsorted && enfr == nfronts &&
              std::equal(eorder.begin(), eorder.end(), order) &&
              std::equal(efs.begin(), efs.end(), fstart);
        printf("order == reference golden: %s\n", eok ? "yes" : "NO");
    }
    free(dwv);
    free(valid);
    free(genes);
    free(order);
    free(fstart);
    free(rank);
    return ok && eok ? 0 : 1;
}
