// eegnet_kernels.hip -- MI355X (gfx950, CDNA4) EEGNet train / infer step behind include/eegnet_abi.h.
//
// Reference being replaced (PraKesEy/EEGNetReplication, /root/reference):
//   EEGNet layers         src/eegnet_repl/model.py:22-84, forward model.py:91-99
//   grad clamps           model.py:43-44 (spatial +-1), 83-84 (classifier +-0.25)
//   CE loss / Adam        train.py:94-103, hot loop model.py:136-148
//
// Algorithm.  The reference materialises the [B,F1,C,T] temporal-conv tensor
// (738 MB at B=4096) and spends 58 % of its step in that conv's weight gradient.  This build never
// forms it.  Everything before the first nonlinearity is linear, so per trial:
//     s[o,t]  = sum_c ws[o,c] x[c,t]                       (spatial first; MFMA f32 16x16x4)
//     v[o,t]  = sum_k w1[o/D,k] s[o,t+k-P]                 (32-tap FIR on F2 rows, not F1*C)
//     y2[o,t] = a1[g] v[o,t] + c1[g] sum_c ws[o,c]         (BN1 affine folded: a1 = g1/sd1)
// BN1's batch statistics come from the lag-Gram of x and window sums; BN2's from sum v, sum v^2.
// Every backward weight-gradient reduction is linear in dy2 and is written as per-trial partial sums
// that finalize code combines with the BN constants at the end.  Five streaming passes (A..E); each
// ends in a ticketed deterministic fp64 reduction whose last workgroup runs the pass's finalize:
//   A  x -> lag-Gram / edge / window sums of x, sum v, sum v^2              (BN1, BN2 statistics)
//   B  x -> v -> BN2 -> ELU -> pool4 -> dropout -> d2, dw16, pw -> sum r, r^2 (BN3 statistics)
//   C  d2 -> block2 -> BN3 -> ELU -> pool8 -> dropout -> FC -> logits [-> CE, dFC, BN3-bwd sums]
//   D  d2 -> block2 bwd (dW3, dw2), dp2, BN2-bwd sums (via pooled ELU' sums E1/E2 stored by B)
//   E  x -> v, dy2 -> dW1 correlation sums, FIR^T(dy2) -> dws GEMM (MFMA)
// All fp32 arithmetic; BN/gradient totals in fp64.  No hipify, no dual paths: gfx950 only.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <stdarg.h>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/eegnet_abi.h"
#include "eegnet_common.h"
#include "eegnet_finalize.hip"
#include "eegnet_stream.hip"
#include "eegnet_passes.hip"
#include "eegnet_wide.hip"
#include "eegnet_infer_bf16.hip"
#include "eegnet_infer_bf16c.hip"
#include "eegnet_host.hip"
