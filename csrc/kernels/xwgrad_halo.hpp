// Patch-reuse weight gradient of the narrow stages' 3x3 stride-1 convs (xwgrad_halo.hip),
// called by xwgrad.hip's dba_xwgrad for the shapes it takes.
#pragma once
#include <hip/hip_runtime.h>

struct XWHArgs {
  const float* dy; long long dy_gstride;   // [G][N][H][W][C]
  const float* x; long long x_gstride;     // [G][N][H][W][C] (lazy: the BN input y)
  float* ws;                               // slabs [Z][G][C][9][C], Z = N * H * W / rows
  const int* nvalid;
  int N, H;
  const int* amax_dy; int amax_dy_ld;      // fp16-pair operand maxima (common.hpp slots)
  const int* amax_x; int amax_x_ld;
  const float* x_coef; int x_relu;         // lazy x: relu?(fma(y, scale, shift)) (bnfuse.hpp rows)
};

// rows (output pixels) per slab for a W x W, Cin -> Cout 3x3 stride-1 conv, 0 = not handled
int xwgrad_halo_rows(int H, int W, int Cin, int Cout);
// -100: not handled (the caller runs the implicit-GEMM weight gradient with the same slabs)
int xwgrad_halo_launch(const XWHArgs& a, int G, int W, int C, hipStream_t st);
