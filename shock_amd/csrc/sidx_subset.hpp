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
// control words of one subset build, kept on the device (the host reads them once, at the end)
enum SubCtl : int {
  SC_FIRSTBAD = 0,  // min over failing ids of (rank << 3 | SubStatus), ~0: none
  SC_SIZE = 1,      // oSize
  SC_K = 2,         // non-blank ids
  SC_KE = 3,        // ids accepted before the first failing one
  SC_NSTART = 4,    // runs among them
  SC_FLAGS = 5,     // 1: rows_cap < Ke, 2: runs_cap < runs, 4: out_cap < the gathered bytes
  SC_TOTAL = 6,     // gathered bytes
  SC_NWORDS = 8,
  // oSize is summed into SC_SLOTS slots past the control words, one per group of workgroups
  // (6,000 workgroups adding into one word at C4 took most of k_sub_runs' 78 us); the host adds them
  SC_SLOTS = 64,
  SC_ALLWORDS = SC_NWORDS + SC_SLOTS
};
#ifndef SIDX_GB_BLOCK
#define SIDX_GB_BLOCK 32768
#endif
constexpr unsigned GATHER_BLOCK = SIDX_GB_BLOCK;  // output bytes per k_gather workgroup (the plan's unit)
}  // namespace sidx
