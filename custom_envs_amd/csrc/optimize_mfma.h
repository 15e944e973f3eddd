// Host entry points of the runtime-shape f64 MFMA Optimize-v0 kernel
// (optimize_mfma.hip; the kernel itself is optimize_mfma_kernel.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "optimize_kernels.h"

namespace ce {

constexpr int kGenMaxF = 64;     // F <= 64: 4 feature tiles of 16
constexpr int kGenMaxClasses = 16;

// Bytes of one [Npad][RS] float64 dataset image row and the padded row count.
int gen_stride_of(int n_features);
int gen_rows_padded_of(int n_rows);
// Raise the dynamic-LDS limit of every instance (double-buffered row blocks).
int gen_set_lds_limits();
void gen_launch_step(const StepArgs<double> &a, hipStream_t stream);
void gen_launch_reset(const StepArgs<double> &a, hipStream_t stream);
// The instance gen_launch_step runs for this shape (as rocprof names it)
std::string gen_kernel_name(int n_envs, int n_rows, int batch, int n_features, int n_classes,
                            int gen_cat);

// Two-class, full-batch, F <= 16 (optimize_lr_mfma.h): 16 envs per workgroup
// on the MFMA N dimension.  The dataset image is fragment-ordered
// (lr_build_image); lr_image_doubles gives its size.
bool lr_shape_ok(int n_features, int n_classes);
size_t lr_image_doubles(int n_features, int n_rows);
void lr_build_image(int n_features, int n_rows, const double *features, const int32_t *labels,
                    double *image);
void lr_launch_step(const StepArgs<double> &a, hipStream_t stream);
// The instance lr_launch_step runs for this shape, as rocprof names it:
// "optimize_lr_mfma_kernel<NKF,MODE,W>"
std::string lr_kernel_name(int n_envs, int n_rows, int n_features, int lr_waves, int mode_cap);

// K steps in one launch (optimize_lr_persist.h, optimize_lr_persist.hip):
// the same two-class full-batch shapes with N <= 512 rows.  Step t reads
// actions a.act + t * act_stride and writes its outputs out_step bytes past
// step t - 1's (0: every step into the same record).
bool lr_persist_ok(int n_rows);
void lr_launch_persist(const StepArgs<double> &a, int k, long long act_stride, long long out_step,
                       hipStream_t stream);
// "optimize_lr_persist_kernel<NKF,TPW,PAD>"
std::string lr_persist_name(int n_rows, int n_features);

}  // namespace ce
