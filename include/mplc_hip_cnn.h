/*
 * mplc_hip_cnn.h - batched multi-model CNN trainer entry points (part of the mplc_hip.h C ABI).
 * Populated as the trainer kernels land; see mplc_hip.h for conventions.
 */
#ifndef MPLC_HIP_CNN_H
#define MPLC_HIP_CNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifdef __cplusplus
}
#endif

#endif /* MPLC_HIP_CNN_H */
