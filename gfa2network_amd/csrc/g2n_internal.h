// g2n_internal.h — host-side plumbing shared by g2n_pipeline.hip and g2n_host.cpp.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/g2n.h"

namespace g2n {

// Internal failure carrying a G2N_E_* status and a message for g2n_last_error().
struct Failure : std::runtime_error {
  int status;
  Failure(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

void set_last_error(const std::string& msg);

// Host-side result storage: g2n_result plus the vectors its pointers refer to.
struct HostResult {
  g2n_result r;
  std::vector<uint8_t> detail, blob, rows, cols, indptr, indices, data;
  std::vector<int64_t> offs;
};

HostResult* new_host_result();
void fill_defaults(g2n_result* r);

// Runs the GPU pipeline on a host buffer (copied to HBM) and downloads the outputs.
int build_host(const void* buf, size_t len, const g2n_options* opts, g2n_result** out, double read_ms);

}  // namespace g2n
