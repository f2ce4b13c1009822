// Host check of rray_amd/csrc/host_libm.inc against the host's glibc (tests/test_host_libm.py).
// Prints one line per function: name, inputs, results that differ, results that differ by more than one ulp.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../rray_amd/csrc/host_libm.inc"

static uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
template <class F, class G, class Gen>
static void run(const char* name, F mine, G libm, Gen gen, int n) {
    std::mt19937_64 rng(20261017);
    long diff = 0, far = 0;
    for (int i = 0; i < n; i++) {
        double x = gen(rng), a = mine(x), b = libm(x);
        if (bits(a) == bits(b) || (a != a && b != b)) continue;
        diff++;
        int64_t d = (int64_t)(bits(a) - bits(b));
        if (d > 1 || d < -1) far++;
    }
    printf("%s %d %ld %ld\n", name, n, diff, far);
}
int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000000;
    auto uni = [](double lo, double hi) {
        return [=](std::mt19937_64& r) { return std::uniform_real_distribution<double>(lo, hi)(r); };
    };
    auto logu = [](double e0, double e1) {
        return [=](std::mt19937_64& r) {
            double m = std::pow(10.0, std::uniform_real_distribution<double>(e0, e1)(r));
            return (r() & 1) ? m : -m;
        };
    };
    auto near_one = [](std::mt19937_64& r) {
        double e = std::pow(10.0, std::uniform_real_distribution<double>(-17, 0)(r));
        return (r() & 1) ? 1 - e : -1 + e;
    };
    auto any_bits = [](std::mt19937_64& r) {
        uint64_t u = r();
        double x;
        memcpy(&x, &u, 8);
        return x;
    };
    run("cbrt", [](double x) { return rrm::cbrt_g(x); }, [](double x) { return std::cbrt(x); }, logu(-300, 300), n);
    run("cbrt_bits", [](double x) { return rrm::cbrt_g(x); }, [](double x) { return std::cbrt(x); }, any_bits, n);
    run("cos", [](double x) { return rrm::cos_g(x); }, [](double x) { return std::cos(x); }, uni(-4, 4), n);
    run("sin", [](double x) { return rrm::sin_g(x); }, [](double x) { return std::sin(x); }, uni(-1.1, 1.1), n);
    run("acos", [](double x) { return rrm::acos_g(x); }, [](double x) { return std::acos(x); }, uni(-1, 1), n);
    run("acos_ends", [](double x) { return rrm::acos_g(x); }, [](double x) { return std::acos(x); }, near_one, n);
    run("atan", [](double x) { return rrm::atan_g(x); }, [](double x) { return std::atan(x); }, logu(-20, 20), n);
    // special values: zeros, infinities, NaN, domain edges
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.5, -0.5, INFINITY, -INFINITY, NAN, 1e-310, -1e-310, 8.0, -27.0,
                         1.7976931348623157e308, 4.9e-324};
    long bad = 0;
    for (double x : sp) {
        double pairs[5][2] = {{rrm::cbrt_g(x), std::cbrt(x)}, {rrm::atan_g(x), std::atan(x)},
                              {rrm::acos_g(x), std::acos(x)}, {rrm::cos_g(x), std::cos(x)}, {rrm::sin_g(x), std::sin(x)}};
        for (auto& p : pairs)
            if (bits(p[0]) != bits(p[1]) && !(p[0] != p[0] && p[1] != p[1])) bad++;
    }
    printf("special %d %ld %ld\n", (int)(sizeof(sp) / sizeof(sp[0])) * 5, bad, bad);
}
