// Host-code sanitizer driver (ASan + UBSan, CPU only; no GPU call succeeds
// here): every host-only C-ABI entry point with realistic and edge shapes,
// and every entry point's argument validation with bad arguments.  The
// draws are printed (one line per array, hex float bits / ints) so the
// pytest wrapper (tests/test_sanitize.py) compares them with the numpy
// oracle; any sanitizer report aborts the process with a non-zero status.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "custom_envs_amd.h"

static int failures = 0;
#define EXPECT(cond)                                                          \
    do {                                                                      \
        if (!(cond)) {                                                        \
            std::fprintf(stderr, "EXPECT failed: %s (line %d)\n", #cond, __LINE__); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

template <typename T> static void dump(const char *tag, const std::vector<T> &v) {
    std::printf("%s", tag);
    for (const T &x : v) {
        uint64_t bits = 0;
        std::memcpy(&bits, &x, sizeof(T));
        std::printf(" %llx", static_cast<unsigned long long>(bits));
    }
    std::printf("\n");
}

int main() {
    EXPECT(ce_abi_version() == CE_ABI_VERSION);
    // ---- host-only draws: edge seeds and shapes
    const uint64_t seeds[] = {0ull, 3ull, 2147483647ull, 8589934592ull, 18446744073709551615ull};
    for (uint64_t s : seeds) {
        std::vector<double> w(10 * 2);
        std::vector<int32_t> p(256);
        EXPECT(ce_seed_draws(s, 10, 2, 256, w.data(), p.data()) == CE_OK);
        std::printf("seed %llu\n", static_cast<unsigned long long>(s));
        dump("lr_w", w);
        dump("lr_p", p);
        const int F = 24, H = 64, K = 10, N = 200;
        std::vector<float> wm(F * H + H + H * K + K);
        std::vector<int32_t> pm(N);
        EXPECT(ce_seed_draws_mlp(s, F, H, K, N, wm.data(), pm.data()) == CE_OK);
        dump("mlp_w", wm);
        dump("mlp_p", pm);
        const int32_t dims[] = {4, 32, 3};
        const int P = 4 * 32 + 32 + 32 * 3 + 3;
        std::vector<float> wn(P);
        std::vector<int32_t> rp(150), ep(150);
        EXPECT(ce_nn_seed_draws(s, 3, dims, 150, wn.data(), rp.data(), ep.data()) == CE_OK);
        dump("nn_w", wn);
        dump("nn_rp", rp);
        dump("nn_ep", ep);
        EXPECT(ce_nn_seed_draws(s, 3, dims, 150, nullptr, nullptr, ep.data()) == CE_OK);
    }
    {   // one row, a large permutation
        std::vector<double> w(3 * 3);
        std::vector<int32_t> p(1);
        EXPECT(ce_seed_draws(7, 3, 3, 1, w.data(), p.data()) == CE_OK && p[0] == 0);
        std::vector<int32_t> big(1 << 20);
        std::vector<double> w2(64 * 16);
        EXPECT(ce_seed_draws(9, 64, 16, 1 << 20, w2.data(), big.data()) == CE_OK);
        std::vector<char> seen(big.size(), 0);
        for (int32_t r : big) EXPECT(r >= 0 && r < (1 << 20) && !seen[r]++);
    }
    // ---- argument validation: every entry point rejects what it must,
    // with a message, and never dereferences a null engine
    EXPECT(ce_seed_draws(1, 0, 2, 10, nullptr, nullptr) == CE_EINVAL);
    EXPECT(ce_seed_draws_mlp(1, 4, 0, 3, 10, nullptr, nullptr) == CE_EINVAL);
    EXPECT(ce_create(nullptr, nullptr, nullptr, nullptr) == CE_EINVAL);
    EXPECT(std::strlen(ce_last_error()) > 0);
    std::vector<double> X(16 * 128, 0.5);
    std::vector<int32_t> y(128, 1);
    ce_engine *eng = nullptr;
    ce_config cfg{};
    cfg.abi_version = CE_ABI_VERSION + 1;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EINVAL && eng == nullptr);
    cfg.abi_version = CE_ABI_VERSION;
    cfg.num_envs = 2;
    cfg.n_rows = 128;
    cfg.n_features = 16;
    cfg.n_classes = 10;
    cfg.batch_size = 129;                       // > n_rows
    cfg.max_steps = 40;
    cfg.precision = CE_F64;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EINVAL);
    cfg.batch_size = 32;
    cfg.max_steps = 0;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EINVAL);
    cfg.max_steps = 40;
    y[5] = 10;                                  // label out of range
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EINVAL);
    y[5] = 1;
    cfg.n_features = 65;                        // past the f64 MFMA kernel's F <= 64
    std::vector<double> X65(65 * 128, 0.5);
    EXPECT(ce_create(&cfg, X65.data(), y.data(), &eng) == CE_EUNSUPPORTED);
    // the network path's geometry checks (net_geometry) run before any HIP call
    cfg.n_features = 16;
    cfg.problem = CE_PROBLEM_MLP;
    cfg.precision = CE_F32;
    cfg.n_layers = 2;
    cfg.hidden[0] = 9000;                       // past the wide-layer path's 8192 units
    cfg.hidden[1] = 64;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EUNSUPPORTED);
    cfg.hidden[0] = 0;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EINVAL);
    cfg.hidden[0] = 64;
    cfg.n_classes = 33;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EUNSUPPORTED);
    cfg.n_classes = 10;
    cfg.n_layers = 5;
    EXPECT(ce_create(&cfg, X.data(), y.data(), &eng) == CE_EUNSUPPORTED);
    // null engines everywhere
    EXPECT(ce_num_envs(nullptr) == CE_EINVAL);
    EXPECT(ce_set_stream(nullptr, nullptr) == CE_EINVAL);
    EXPECT(ce_set_compact_outputs(nullptr, 1) == CE_EINVAL);
    EXPECT(ce_seed(nullptr, nullptr, 0) == CE_EINVAL);
    EXPECT(ce_reset(nullptr, nullptr, 0) == CE_EINVAL);
    EXPECT(ce_step(nullptr, nullptr, nullptr, 0) == CE_EINVAL);
    EXPECT(ce_step_many(nullptr, 4, nullptr, 0, nullptr) == CE_EINVAL);
    EXPECT(ce_get_state(nullptr, nullptr) == CE_EINVAL);
    EXPECT(ce_set_state(nullptr, nullptr) == CE_EINVAL);
    EXPECT(ce_host_outputs(nullptr, nullptr) == CE_EINVAL);
    EXPECT(std::strcmp(ce_step_kernel(nullptr), "") == 0);
    ce_destroy(nullptr);
    EXPECT(ce_multi_create(nullptr, nullptr) == CE_EINVAL);
    ce_multi_destroy(nullptr);
    EXPECT(ce_nn_create(nullptr, nullptr, nullptr, nullptr) == CE_EINVAL);
    ce_nn_destroy(nullptr);
    std::printf("failures %d\n", failures);
    return failures ? 1 : 0;
}
