// Host-side seeding: gym.utils.seeding.np_random restated natively.
//
// Reference call sites: BaseEnvironment.seed (custom_envs/envs/
// baseenvironment.py:20-28) and the draws every reset replays under
// use_random_state (custom_envs/utils/utils_math.py:9-22):
// ModelNumpy.reset -> npr.normal(size=(F, K)) and InMemoryDataSet.shuffle ->
// npr.shuffle(arange(N)) (custom_envs/utils/utils_common.py:12-23), in that
// order (optimize.py:63-64).
//
// Third-party algorithms restated (published, pinned by tests against
// hashlib + numpy.random.RandomState):
//   gym<=0.21 hash_seed:   sha512(str(seed))[:8] as little-endian u32 words
//   numpy MT19937:         init_by_array, genrand_int32, res53 doubles
//   numpy legacy_gauss:    Marsaglia polar method with one cached value
//   numpy legacy shuffle:  Fisher-Yates from the top with masked rejection
//                          sampling (random_interval)
#include "seeding.h"

#include <cmath>
#include <cstdio>
#include <cstring>

#include <algorithm>
#include <vector>

namespace ce {
namespace {

// ---------------------------------------------------------------- SHA-512
constexpr uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL,
    0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL,
    0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL,
    0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL,
    0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL, 0x2de92c6f592b0275ULL,
    0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL,
    0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL,
    0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL,
    0x92722c851482353bULL, 0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL,
    0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL,
    0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL,
    0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL,
    0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL,
    0xc67178f2e372532bULL, 0xca273eceea26619cULL, 0xd186b8c721c0c207ULL,
    0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL,
    0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL,
    0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// One-shot SHA-512 of a short message (< 112 bytes: one padded block).
void sha512_short(const uint8_t *msg, size_t len, uint8_t out[64]) {
    uint8_t block[128] = {0};
    std::memcpy(block, msg, len);
    block[len] = 0x80;
    const uint64_t bits = static_cast<uint64_t>(len) * 8;
    for (int i = 0; i < 8; ++i) block[127 - i] = static_cast<uint8_t>(bits >> (8 * i));
    uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                     0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                     0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                     0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint64_t w[80];
    for (int t = 0; t < 16; ++t) {
        uint64_t v = 0;
        for (int b = 0; b < 8; ++b) v = (v << 8) | block[8 * t + b];
        w[t] = v;
    }
    for (int t = 16; t < 80; ++t) {
        const uint64_t s0 = rotr(w[t - 15], 1) ^ rotr(w[t - 15], 8) ^ (w[t - 15] >> 7);
        const uint64_t s1 = rotr(w[t - 2], 19) ^ rotr(w[t - 2], 61) ^ (w[t - 2] >> 6);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 80; ++t) {
        const uint64_t S1 = rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41);
        const uint64_t ch = (e & f) ^ (~e & g);
        const uint64_t t1 = hh + S1 + ch + kSha512K[t] + w[t];
        const uint64_t S0 = rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39);
        const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint64_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    for (int i = 0; i < 8; ++i)
        for (int b2 = 0; b2 < 8; ++b2) out[8 * i + b2] = static_cast<uint8_t>(h[i] >> (56 - 8 * b2));
}

}  // namespace

int seed_key(uint64_t seed, uint32_t key[2]) {
    char text[32];
    const int len = std::snprintf(text, sizeof(text), "%llu",
                                  static_cast<unsigned long long>(seed));
    uint8_t digest[64];
    sha512_short(reinterpret_cast<const uint8_t *>(text), static_cast<size_t>(len), digest);
    uint32_t w[2];
    for (int i = 0; i < 2; ++i)
        w[i] = static_cast<uint32_t>(digest[4 * i]) |
               (static_cast<uint32_t>(digest[4 * i + 1]) << 8) |
               (static_cast<uint32_t>(digest[4 * i + 2]) << 16) |
               (static_cast<uint32_t>(digest[4 * i + 3]) << 24);
    // _int_list_from_bigint: base-2**32 digits, no leading zero digits,
    // [0] for zero.
    key[0] = w[0];
    key[1] = w[1];
    return w[1] != 0 ? 2 : 1;
}

void Mt19937::init_by_array(const uint32_t *key, int n) {
    mt[0] = 19650218u;
    for (int i = 1; i < kN; ++i)
        mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    int i = 1, j = 0;
    for (int k = (kN > n ? kN : n); k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] +
                static_cast<uint32_t>(j);
        ++i; ++j;
        if (i >= kN) { mt[0] = mt[kN - 1]; i = 1; }
        if (j >= n) j = 0;
    }
    for (int k = kN - 1; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) -
                static_cast<uint32_t>(i);
        ++i;
        if (i >= kN) { mt[0] = mt[kN - 1]; i = 1; }
    }
    mt[0] = 0x80000000u;
    pos = kN;
    has_gauss = false;
    gauss = 0.0;
}

void Mt19937::generate() {
    constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
    int k = 0;
    for (; k < kN - kM; ++k) {
        const uint32_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
        mt[k] = mt[k + kM] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    }
    for (; k < kN - 1; ++k) {
        const uint32_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
        mt[k] = mt[k + (kM - kN)] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    }
    const uint32_t y = (mt[kN - 1] & kUpper) | (mt[0] & kLower);
    mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    pos = 0;
}

uint32_t Mt19937::next32() {
    if (pos >= kN) generate();
    uint32_t y = mt[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double Mt19937::next_double() {
    const uint32_t a = next32() >> 5, b = next32() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

double Mt19937::next_gauss() {
    if (has_gauss) {
        has_gauss = false;
        const double cached = gauss;
        gauss = 0.0;
        return cached;
    }
    double x1, x2, r2;
    do {
        x1 = 2.0 * next_double() - 1.0;
        x2 = 2.0 * next_double() - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    gauss = f * x1;
    has_gauss = true;
    return f * x2;
}

uint64_t Mt19937::interval(uint64_t max) {
    if (max == 0) return 0;
    uint64_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    uint64_t value;
    if (max <= 0xffffffffULL) {
        while ((value = (next32() & mask)) > max) {}
    } else {
        while ((value = (((static_cast<uint64_t>(next32()) << 32) | next32()) & mask)) > max) {}
    }
    return value;
}

void reset_draws(uint64_t seed, int n_features, int n_classes, int n_rows,
                 double *init_weights, int32_t *perm) {
    uint32_t key[2];
    const int key_len = seed_key(seed, key);
    Mt19937 rng;
    rng.init_by_array(key, key_len);
    const int n_params = n_features * n_classes;
    for (int i = 0; i < n_params; ++i) {
        const double v = rng.next_gauss();
        if (init_weights) init_weights[i] = v;
    }
    if (!perm) return;
    for (int i = 0; i < n_rows; ++i) perm[i] = i;
    for (int i = n_rows - 1; i > 0; --i) {
        const int j = static_cast<int>(rng.interval(static_cast<uint64_t>(i)));
        const int32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
}

static void legacy_shuffle(Mt19937 &rng, int n_rows, int32_t *perm) {
    for (int i = 0; i < n_rows; ++i) perm[i] = i;
    for (int i = n_rows - 1; i > 0; --i) {
        const int j = static_cast<int>(rng.interval(static_cast<uint64_t>(i)));
        const int32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
}

void reset_draws_net(uint64_t seed, int n_dims, const int *dims, int n_rows, float *init_weights,
                     int32_t *perm) {
    uint32_t key[2];
    const int key_len = seed_key(seed, key);
    Mt19937 rng;
    rng.init_by_array(key, key_len);
    // RandomState.uniform(low, high): low + (high - low) * random_sample(),
    // layer by layer in trainable_variables order, biases zero
    size_t off = 0;
    for (int l = 0; l + 1 < n_dims; ++l) {
        const int fan_in = dims[l], fan_out = dims[l + 1];
        const double limit = std::sqrt(6.0 / static_cast<double>(fan_in + fan_out));
        const double low = -limit, range = limit - low;
        const size_t n = static_cast<size_t>(fan_in) * fan_out;
        for (size_t i = 0; i < n; ++i) {
            const double v = low + range * rng.next_double();
            if (init_weights) init_weights[off + i] = static_cast<float>(v);
        }
        off += n;
        if (init_weights)
            for (int i = 0; i < fan_out; ++i) init_weights[off + i] = 0.0f;
        off += fan_out;
    }
    // then sequence.shuffle() on the same stream (optimize.py:63-64)
    if (perm) legacy_shuffle(rng, n_rows, perm);
}

void reset_draws_mlp(uint64_t seed, int n_features, int n_hidden, int n_classes, int n_rows,
                     float *init_weights, int32_t *perm) {
    const int dims[3] = {n_features, n_hidden, n_classes};
    reset_draws_net(seed, 3, dims, n_rows, init_weights, perm);
}

}  // namespace ce

namespace ce {

void reset_draws_nn(uint64_t seed, int n_dims, const int *dims, int n_rows, float *init_weights,
                    int32_t *reset_perm, int32_t *epoch_perm) {
    uint32_t key[2];
    const int key_len = seed_key(seed, key);
    Mt19937 rng;
    rng.init_by_array(key, key_len);
    size_t off = 0;
    for (int l = 0; l + 1 < n_dims; ++l) {
        const int fan_in = dims[l], fan_out = dims[l + 1];
        const double limit = std::sqrt(6.0 / static_cast<double>(fan_in + fan_out));
        const double low = -limit, range = limit - low;
        const size_t n = static_cast<size_t>(fan_in) * fan_out;
        for (size_t i = 0; i < n; ++i) {
            const double v = low + range * rng.next_double();
            if (init_weights) init_weights[off + i] = static_cast<float>(v);
        }
        off += n;
        if (init_weights)
            for (int i = 0; i < fan_out; ++i) init_weights[off + i] = 0.0f;
        off += fan_out;
    }
    // The kernels stand in for TF's RNG, which is not numpy's: the reset's
    // shuffle (OptimizeNN.reset -> next() -> on_epoch_end, optimize_nn.py:
    // 102-120) is the first draw of the fresh env stream, the same
    // permutation every epoch end inside a step draws.
    if (reset_perm || epoch_perm) {
        Mt19937 fresh;
        fresh.init_by_array(key, key_len);
        std::vector<int32_t> perm(n_rows);
        legacy_shuffle(fresh, n_rows, perm.data());
        if (reset_perm) std::copy(perm.begin(), perm.end(), reset_perm);
        if (epoch_perm) std::copy(perm.begin(), perm.end(), epoch_perm);
    }
}

}  // namespace ce
