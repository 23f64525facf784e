// sidx_subset.hpp -- status codes shared by the subset kernels and the C ABI.
#pragma once
namespace sidx {
// per-id outcome, in the order subset.go:201-223 checks them
enum SubStatus : unsigned {
  SUB_OK = 0,
  SUB_SYNTAX = 1,  // strconv.Atoi: parsing "...": invalid syntax
  SUB_RANGE = 2,   // strconv.Atoi: parsing "...": value out of range
  SUB_SORT = 3,    // Subset indices must be numerically sorted and non-redundant, ...
  SUB_EXIST = 4,   // Subset index: %d does not exist in parent index file.
  SUB_READ = 5,    // Subset index could not read parent index file for part: %d
};
}  // namespace sidx
