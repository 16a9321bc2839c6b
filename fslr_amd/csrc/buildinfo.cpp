// buildinfo.cpp — the hash of the kernel sources this libfslr_hip.so was built from (Makefile:
// sha256 of the sorted *.hip / *.hpp of this directory, then include/fslr_hip.h, first 16 hex
// digits).  fslr_amd/_lib.py computes the same over the sources beside it and refuses a stale
// binary.
#ifndef FSLR_SRC_HASH
#define FSLR_SRC_HASH "unknown"
#endif

extern "C" const char* fslr_source_hash(void) { return FSLR_SRC_HASH; }
