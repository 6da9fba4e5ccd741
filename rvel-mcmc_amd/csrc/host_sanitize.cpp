// Host-side sanitizer driver for librvmcmc's C ABI (not part of the library): every entry point's
// argument checks, and rvm_plan_create's host work (epoch split, sort, segment schedule, weights)
// on valid inputs -- the first HIP call then fails on a GPU-less host, which is an error return.
// Built with AddressSanitizer + UBSan on the host side only (`make sanitize-host`), run by
// tests/test_sanitizers.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/rvmcmc.h"

int main() {
    int fails = 0;
    auto expect = [&](bool ok, const char* what) {
        if (!ok) {
            std::fprintf(stderr, "FAIL %s\n", what);
            fails++;
        }
    };
    expect(rvm_abi_version() == RVM_ABI_VERSION, "abi version");
    rvm_config cfg{};
    cfg.n_planets = 2;
    cfg.dt = 0.65;
    cfg.n_levels = 4;
    cfg.npoints_norm = 100.0;
    const int mult[4] = {4, 5, 6, 7};
    std::memcpy(cfg.level_mult, mult, sizeof(mult));
    cfg.period_hint = 5.2;
    std::vector<double> t, rv, sg;
    for (int i = 0; i < 101; i++) {  // both directions, unsorted, a duplicate epoch
        t.push_back(i % 2 ? -0.6 * i : 0.55 * (100 - i));
        rv.push_back(1e-4 * std::sin(i));
        sg.push_back(1.5e-4);
    }
    t[7] = t[9];
    rvm_plan* plan = nullptr;
    const int rc = rvm_plan_create(&cfg, t.data(), rv.data(), sg.data(), (int)t.size(), 4096, &plan);
    expect(rc == 0 || (rc < 0 && plan == nullptr), "plan_create valid input");
    if (rc == 0) rvm_plan_destroy(plan);
    rvm_config bad = cfg;
    bad.n_levels = 0;
    expect(rvm_plan_create(&bad, t.data(), rv.data(), sg.data(), (int)t.size(), 64, &plan) < 0, "n_levels 0");
    bad = cfg;
    bad.level_mult[1] = 4;
    expect(rvm_plan_create(&bad, t.data(), rv.data(), sg.data(), (int)t.size(), 64, &plan) < 0, "dup multipliers");
    bad = cfg;
    bad.dt = -1.0;
    expect(rvm_plan_create(&bad, t.data(), rv.data(), sg.data(), (int)t.size(), 64, &plan) < 0, "negative dt");
    std::vector<double> tn = t;
    tn[3] = NAN;
    expect(rvm_plan_create(&cfg, tn.data(), rv.data(), sg.data(), (int)t.size(), 64, &plan) < 0, "nan epoch");
    expect(std::strlen(rvm_last_error()) > 0, "last_error");
    expect(rvm_logl_batch(nullptr, 1, nullptr, 1.0, nullptr, nullptr, nullptr, nullptr) < 0, "logl null plan");
    rvm_param_map pm{};
    expect(rvm_stretch_half_step(nullptr, &pm, 10, 1, 0, nullptr, nullptr, nullptr, 1, nullptr, 2.0, 0, 0, 0, 1.0,
                                 nullptr, nullptr, nullptr, nullptr) < 0,
           "half_step null plan");
    expect(rvm_stretch_propose(0, 1, 0, nullptr, 1, nullptr, 2.0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr) < 0,
           "propose bad");
    expect(rvm_mh_accept(0, 1, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr) < 0, "mh bad");
    expect(rvm_fd_params(10, 1, nullptr, 1e-6, nullptr, nullptr, nullptr) < 0, "fd bad");
    const int32_t rows[2] = {0, 0};
    expect(rvm_logl_derivs(nullptr, 1, nullptr, 2, rows, 1.0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) < 0,
           "derivs null plan");
    expect(rvm_logl_derivs_workspace_bytes(256, 10) == (size_t)256 * 55 * 2 * 36, "derivs workspace");
    rvm_smala_cache c{};
    expect(rvm_smala_metric(10, 1, nullptr, nullptr, nullptr, nullptr, nullptr, 1.0, 0.5, &c, nullptr) < 0, "metric bad");
    std::printf("host sanitize driver: %d failures\n", fails);
    return fails;
}
