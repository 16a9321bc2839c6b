// Test driver for the BAM decoder under AddressSanitizer (tests/test_bam.py::test_corrupt_bam_*):
// opens every path given, decodes the columns and every record's sequence, and prints one line per
// file: "ok <records>" or "error".  Any out-of-bounds access aborts the process (ASan).
#include <cstdio>
#include <string>
#include <vector>

#include "fslr_bam.h"

int main(int argc, char **argv) {
  for (int k = 1; k < argc; ++k) {
    FslrBam *b = nullptr;
    char err[256] = {0};
    if (fslr_bam_open(argv[k], 2, &b, err, sizeof(err)) != FSLR_BAM_OK) {
      std::printf("error open\n");
      continue;
    }
    const int64_t n = fslr_bam_n_records(b);
    std::vector<int32_t> flag(n), tid(n), mapq(n), ncig(n);
    std::vector<int64_t> pos(n), span(n), rlen(n), c0(n), c1(n), as(n), ls(n), qe(n);
    std::vector<int8_t> ak(n);
    std::vector<char> qn(static_cast<size_t>(fslr_bam_qname_bytes(b)) + 1);
    int rc = fslr_bam_columns(b, flag.data(), tid.data(), pos.data(), mapq.data(), span.data(), rlen.data(), c0.data(),
                              c1.data(), ncig.data(), as.data(), ak.data(), ls.data(), qe.data(), qn.data());
    for (int64_t r = 0; rc == FSLR_BAM_OK && r < n; ++r) {
      std::string s(static_cast<size_t>(ls[r]) + 1, '\0');
      rc = fslr_bam_forward_seq(b, r, &s[0]);
    }
    std::printf(rc == FSLR_BAM_OK ? "ok %lld\n" : "error columns\n", static_cast<long long>(n));
    fslr_bam_close(b);
  }
  return 0;
}
