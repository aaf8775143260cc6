// `a4 --format mtx` (csr_chain.cpp): the Matrix Market chain on the CSR engine.
#pragma once

#include <string>
#include <vector>

namespace a4 {

struct MtxOptions {
  std::vector<std::string> inputs;   // .mtx files in chain order, or one folder of them
  std::string out = "matrix.mtx", device = "auto", metrics, comm = "auto";
  int threads = 0, local_rank = 0;
  double timeout = 120.0;   // bounded RCCL waits
  bool quiet = false;
};

// Collective over MPI_COMM_WORLD; throws a4::Error on bad input.
int run_mtx(const MtxOptions& o, int rank, int world);

}  // namespace a4
