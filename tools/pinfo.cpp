// Diagnostic: print the engine capacities of a configuration (host only).
//   g++ -std=c++17 -O1 -o /tmp/pinfo tools/pinfo.cpp && /tmp/pinfo 5 5 5
#include <cstdio>
#include <cstdlib>

#include "../optimalcontrolmps_amd/csrc/params.hpp"

int main(int argc, char** argv) {
  const int L = argc > 1 ? std::atoi(argv[1]) : 5, p = argc > 2 ? std::atoi(argv[2]) : 5,
            Q = argc > 3 ? std::atoi(argv[3]) : 5;
  OcgParams P;
  std::vector<int> md;
  std::string e = ocg_host::build_params(P, md, L, p, Q, 0.01, 1e-8, 80);
  if (!e.empty()) { std::printf("error: %s\n", e.c_str()); return 1; }
  std::printf("cap %d thcap %d evcap %d nrot %d ecap %d max_site_cap %d nsq %d\n", P.cap, P.thcap, P.evcap, P.nrot,
              P.ecap, P.max_site_cap, P.nsq);
  for (int k = 1; k <= L; ++k) std::printf("site %d cap %d\n", k, P.site_cap[k]);
  return 0;
}
