// Native restatement of gym<=0.21 np_random + numpy RandomState draws.
#pragma once
#include <cstdint>

namespace ce {

struct Mt19937 {
    static constexpr int kN = 624, kM = 397;
    uint32_t mt[kN];
    int pos = kN;
    bool has_gauss = false;
    double gauss = 0.0;

    void init_by_array(const uint32_t *key, int n);
    void generate();
    uint32_t next32();
    double next_double();
    double next_gauss();
    uint64_t interval(uint64_t max);
};

// Key words RandomState.seed() receives for gym's np_random(seed); returns
// the key length (1 or 2).
int seed_key(uint64_t seed, uint32_t key[2]);

// (W0, perm) drawn by every reset of an env seeded with `seed`: F*K legacy
// gaussians in C order, then a legacy shuffle of arange(n_rows).  Either
// output may be null.
void reset_draws(uint64_t seed, int n_features, int n_classes, int n_rows,
                 double *init_weights, int32_t *perm);

// (W0, perm) of the MLP problem: glorot-uniform W1
// (F x H) then W2 (H x K) as legacy uniform(-l, l) draws rounded to float32,
// zero biases, in the flat order [W1 | b1 | W2 | b2]; then the legacy
// shuffle of arange(n_rows).  Either output may be null.
void reset_draws_mlp(uint64_t seed, int n_features, int n_hidden, int n_classes, int n_rows,
                     float *init_weights, int32_t *perm);
// The same for any depth (dims = F, hidden..., K): every layer's kernel
// glorot-uniform in order, zero biases, then the shuffle on the same stream.
void reset_draws_net(uint64_t seed, int n_dims, const int *dims, int n_rows, float *init_weights,
                     int32_t *perm);

// MultiOptLRs over the OptimizeNN problem (oracle/multinn.py nn_draws):
// glorot-uniform kernels of every layer (dims[0] -> dims[1] -> ...) as legacy
// uniform(-l, l) draws rounded to float32, zero biases, flat order
// [W1 | b1 | W2 | b2 | ...]; then the reset's legacy shuffle of arange(N);
// epoch_perm is the first shuffle of a fresh copy of the seed's stream (the
// one every epoch end inside a step draws).  Any output may be null.
void reset_draws_nn(uint64_t seed, int n_dims, const int *dims, int n_rows, float *init_weights,
                    int32_t *reset_perm, int32_t *epoch_perm);

}  // namespace ce
