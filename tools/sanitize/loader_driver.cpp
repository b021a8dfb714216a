// Host-only driver for the native batch builder (ops/csrc/pbx_loader.cpp) under the compiler
// sanitizers: built with -fsanitize=address,undefined or -fsanitize=thread by
// tests/test_host_sanitizers.py and run on a small .pbxds store.  Exercises open / multi-threaded
// ring production / in-order consumption across epochs / early destroy with workers mid-batch /
// resume from a batch index / error paths.  Prints one checksum line; any sanitizer report fails the run.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
void* pbxl_open(const char* dir, int n_annotations, const uint8_t* lut, char* err, int errlen);
int64_t pbxl_size(void* store);
void pbxl_close(void* store);
void* pbxl_loader_create(void* store, int B, int L, const int64_t* indices, int64_t n_indices, uint64_t seed,
                         int shuffle, int drop_last, int include_last_window, int nthreads, int depth,
                         int64_t start_batch, char* err, int errlen);
int64_t pbxl_batches_per_epoch(void* loader);
int pbxl_next(void* loader, uint8_t* tokens_out, uint8_t* bits_out, int64_t* batch_id_out);
void pbxl_loader_destroy(void* loader);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s store_dir n_annotations\n", argv[0]);
    return 2;
  }
  const int A = std::atoi(argv[2]);
  uint8_t lut[256];
  for (int i = 0; i < 256; ++i) lut[i] = (uint8_t)(3 + i % 25);
  char err[512];
  void* st = pbxl_open(argv[1], A, lut, err, sizeof(err));
  if (!st) {
    std::fprintf(stderr, "open failed: %s\n", err);
    return 1;
  }
  // error path: a missing store reports instead of crashing
  if (pbxl_open("/nonexistent-pbxds", A, lut, err, sizeof(err)) != nullptr) return 1;
  const int64_t n = pbxl_size(st);
  std::vector<int64_t> idx(n);
  for (int64_t i = 0; i < n; ++i) idx[i] = i;
  const int B = 4, L = 64, nbytes = (A + 7) / 8;
  std::vector<uint8_t> tok((size_t)B * L), bits((size_t)B * nbytes);
  uint64_t sum = 0;
  for (int threads : {1, 3, 8}) {
    void* ld = pbxl_loader_create(st, B, L, idx.data(), n, 7, 1, 0, threads & 1, threads, 2, 0, err, sizeof(err));
    if (!ld) {
      std::fprintf(stderr, "create failed: %s\n", err);
      return 1;
    }
    const int64_t nb = pbxl_batches_per_epoch(ld);
    for (int64_t i = 0; i < 3 * nb; ++i) {
      int64_t bid = -1;
      const int rows = pbxl_next(ld, tok.data(), bits.data(), &bid);
      if (rows <= 0 || bid != i) {
        std::fprintf(stderr, "bad batch %lld rows %d id %lld\n", (long long)i, rows, (long long)bid);
        return 1;
      }
      for (size_t k = 0; k < tok.size(); ++k) sum = sum * 31 + tok[k];
      for (size_t k = 0; k < bits.size(); ++k) sum = sum * 131 + bits[k];
    }
    pbxl_loader_destroy(ld);          // workers may be mid-batch filling the ring
  }
  // resume from a batch index, destroyed right after the first batch
  void* ld = pbxl_loader_create(st, B, L, idx.data(), n, 7, 1, 1, 0, 4, 6, 5, err, sizeof(err));
  if (!ld) return 1;
  int64_t bid = -1;
  if (pbxl_next(ld, tok.data(), bits.data(), &bid) <= 0 || bid != 5) return 1;
  pbxl_loader_destroy(ld);
  // invalid arguments are refused
  if (pbxl_loader_create(st, 0, L, idx.data(), n, 7, 1, 0, 0, 1, 1, 0, err, sizeof(err)) != nullptr) return 1;
  int64_t bad = n + 3;
  if (pbxl_loader_create(st, B, L, &bad, 1, 7, 1, 0, 0, 1, 1, 0, err, sizeof(err)) != nullptr) return 1;
  pbxl_close(st);
  std::printf("ok %llu\n", (unsigned long long)sum);
  return 0;
}
