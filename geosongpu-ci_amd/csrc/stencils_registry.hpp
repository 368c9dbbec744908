// stencils_registry.hpp — name -> stencil dispatch for gtfv3_stencil (the
// NDSL-style `stencil(*fields, params)` call surface used by the Python hook
// and the parity tests).  Each entry validates its field list.
#pragma once
#include <string>
#include <vector>

namespace gtfv3 {
class Dycore;
void run_registered_stencil(Dycore& dy, const std::string& name, const std::vector<std::string>& fields,
                            const std::vector<double>& params);
std::vector<std::string> registered_stencils();
}  // namespace gtfv3
