// The fused-twiddle transforms' constant tables (lf512.hpp / lf1k.hpp layouts) as the product builds them
// (client.cpp make_lf512_table / make_lf1k_table) against the oracle's plans (or_lf_table / or_lf1k_table):
// equal bit for bit, which is what makes the device lane programs and the oracle's restatement compute
// the same values.  Built and run by tests/test_native_helpers.py (CPU only).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace tae {
std::vector<double> make_lf512_table();
std::vector<double> make_lf1k_table();
}  // namespace tae

extern "C" {
void *or_lf_plan_new(void);
void *or_lf1k_plan_new(void);
void or_lf_any_free(void *plan);
void or_lf_table(const void *plan, double *t);
void or_lf1k_table(const void *plan, double *t);
}

static int compare(const char *name, const std::vector<double> &got, const std::vector<double> &want) {
    if (got.size() != want.size()) {
        printf("%s: %zu doubles, oracle %zu\n", name, got.size(), want.size());
        return 1;
    }
    int bad = 0;
    for (size_t i = 0; i < got.size(); i++)
        if (std::memcmp(&got[i], &want[i], sizeof(double)) != 0 && bad++ < 5)
            printf("%s[%zu]: %a, oracle %a\n", name, i, got[i], want[i]);
    return bad;
}

int main() {
    void *p = or_lf_plan_new(), *q = or_lf1k_plan_new();
    std::vector<double> t512(1700), t1k(3788);
    or_lf_table(p, t512.data());
    or_lf1k_table(q, t1k.data());
    const int bad = compare("lf512", tae::make_lf512_table(), t512) + compare("lf1k", tae::make_lf1k_table(), t1k);
    or_lf_any_free(p);
    or_lf_any_free(q);
    if (bad) return 1;
    printf("OK\n");
    return 0;
}
