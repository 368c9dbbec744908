// kernels_column.hpp — launchers of the K-column primitives (column.hip).
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

void column_top(const Ctx& c, int nk, const double* in, double* out);
void column_while_lt(const Ctx& c, int nk, double thr, const double* in, double* out);
void column_gather_k(const Ctx& c, int nk, const double* data, const double* kmask, const double* kidx,
                     double* out);

}  // namespace gtfv3
