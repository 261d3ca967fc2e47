// Host-runtime self-test, built by tests/test_native_sanitizers.py with -fsanitize=address,undefined
// and separately with -fsanitize=thread (the CIFAR prefetch ring is the one multi-threaded
// component).  Links the runtime sources directly: no Python, no GPU, no LD_PRELOAD.
// the reference has no sanitizer builds at all; this is the MI355X framework's
// host-side race/memory checking.  Exit 0 and print "runtime selftest OK" on success.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
uint32_t dtm_crc32c(const void* data, size_t n);
uint32_t dtm_crc32c_masked(const void* data, size_t n);
void* dtm_tfrecord_writer_open(const char* path);
int dtm_tfrecord_write(void* h, const void* data, int64_t n);
int dtm_tfrecord_writer_close(void* h);
void* dtm_tfrecord_reader_open(const char* path, int verify);
int64_t dtm_tfrecord_next(void* h, const char** data);
void dtm_tfrecord_reader_close(void* h);
void* dtm_cifar_table_open(const char* files, int label_bytes);
int64_t dtm_cifar_table_size(void* h);
int dtm_cifar_table_get(void* h, int64_t start, int n, uint8_t* images, int32_t* labels);
int dtm_loader_start(void* h, int batch, int nslots, uint8_t* img, int32_t* lab, int shuffle, uint64_t seed);
int dtm_loader_next(void* h);
void dtm_loader_release(void* h, int slot);
void dtm_cifar_table_close(void* h);
void* dtm_bundle_writer_new(const char* prefix);
int dtm_bundle_writer_add(void* h, const char* name, int dtype, const int64_t* shape, int ndim, const void* data,
                          int64_t nbytes);
int dtm_bundle_writer_finish(void* h);
void* dtm_bundle_reader_open(const char* prefix);
int dtm_bundle_reader_num(void* h);
const char* dtm_bundle_reader_name(void* h, int i);
int dtm_bundle_reader_info(void* h, int i, int* dtype, int64_t* shape, int* ndim, int64_t* nbytes);
int dtm_bundle_reader_read(void* h, int i, void* dst, int64_t nbytes);
void dtm_bundle_reader_close(void* h);
}

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

static void test_crc() {
  CHECK(dtm_crc32c("123456789", 9) == 0xE3069283u);  // CRC-32C check value
  std::vector<uint8_t> big(1 << 20);
  for (size_t i = 0; i < big.size(); ++i) big[i] = (uint8_t)(i * 131 + 7);
  // unaligned tails through the hardware/software paths
  for (int off = 0; off < 9; ++off) (void)dtm_crc32c(big.data() + off, big.size() - off - 3);
  (void)dtm_crc32c_masked(big.data(), big.size());
}

static void test_tfrecord(const std::string& dir) {
  std::string path = dir + "/t.tfrecord";
  void* w = dtm_tfrecord_writer_open(path.c_str());
  CHECK(w);
  std::vector<std::string> recs;
  for (int i = 0; i < 50; ++i) {
    recs.emplace_back((size_t)(i * 37 % 4096 + (i == 7 ? 0 : 1)), (char)('a' + i % 26));
    CHECK(dtm_tfrecord_write(w, recs.back().data(), (int64_t)recs.back().size()) == 0);
  }
  CHECK(dtm_tfrecord_writer_close(w) == 0);
  void* r = dtm_tfrecord_reader_open(path.c_str(), 1);
  CHECK(r);
  const char* data = nullptr;
  for (int i = 0; i < 50; ++i) {
    int64_t n = dtm_tfrecord_next(r, &data);
    CHECK(n == (int64_t)recs[i].size());
    CHECK(std::memcmp(data, recs[i].data(), (size_t)n) == 0);
  }
  CHECK(dtm_tfrecord_next(r, &data) < 0);  // clean EOF
  dtm_tfrecord_reader_close(r);
  // corrupt one payload byte: the verifying reader must stop at that record, never read past it
  FILE* f = std::fopen(path.c_str(), "r+b");
  CHECK(f);
  std::fseek(f, 12, SEEK_SET);  // first payload byte of record 0
  std::fputc('#', f);
  std::fclose(f);
  r = dtm_tfrecord_reader_open(path.c_str(), 1);
  CHECK(r);
  CHECK(dtm_tfrecord_next(r, &data) < 0);
  dtm_tfrecord_reader_close(r);
}

static void test_bundle(const std::string& dir) {
  std::string prefix = dir + "/model.ckpt-1";
  void* w = dtm_bundle_writer_new(prefix.c_str());
  CHECK(w);
  std::vector<float> a(3 * 5 * 7);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0.5f * (float)i - 3.f;
  int64_t sa[3] = {3, 5, 7};
  int64_t gs = 1234;
  CHECK(dtm_bundle_writer_add(w, "conv1/weights", 1, sa, 3, a.data(), (int64_t)(a.size() * 4)) == 0);
  CHECK(dtm_bundle_writer_add(w, "global_step", 9, nullptr, 0, &gs, 8) == 0);
  CHECK(dtm_bundle_writer_finish(w) == 0);
  void* r = dtm_bundle_reader_open(prefix.c_str());
  CHECK(r);
  CHECK(dtm_bundle_reader_num(r) == 2);
  for (int i = 0; i < 2; ++i) {
    int dt = 0, nd = 0;
    int64_t shape[8], nb = 0;
    CHECK(dtm_bundle_reader_info(r, i, &dt, shape, &nd, &nb) == 0);
    std::vector<uint8_t> buf((size_t)nb);
    CHECK(dtm_bundle_reader_read(r, i, buf.data(), nb) == 0);
    if (std::string(dtm_bundle_reader_name(r, i)) == "conv1/weights") {
      CHECK(nd == 3 && shape[0] == 3 && shape[2] == 7 && nb == (int64_t)(a.size() * 4));
      CHECK(std::memcmp(buf.data(), a.data(), (size_t)nb) == 0);
    } else {
      CHECK(nb == 8 && std::memcmp(buf.data(), &gs, 8) == 0);
    }
  }
  CHECK(dtm_bundle_reader_info(r, 5, nullptr, nullptr, nullptr, nullptr) < 0);  // out of range
  dtm_bundle_reader_close(r);
}

static void test_cifar_loader(const std::string& dir) {
  std::string p = dir + "/data_batch_1.bin";
  FILE* f = std::fopen(p.c_str(), "wb");
  CHECK(f);
  const int N = 97;
  std::vector<uint8_t> rec(3073);
  for (int i = 0; i < N; ++i) {
    rec[0] = (uint8_t)(i % 10);
    for (int j = 0; j < 3072; ++j) rec[1 + j] = (uint8_t)(i + j);
    std::fwrite(rec.data(), 1, rec.size(), f);
  }
  std::fclose(f);
  void* h = dtm_cifar_table_open(p.c_str(), 1);
  CHECK(h && dtm_cifar_table_size(h) == N);
  std::vector<uint8_t> one(3072 * 2);
  int32_t lab[2];
  CHECK(dtm_cifar_table_get(h, N - 1, 2, one.data(), lab) == 0);  // wraps around
  CHECK(lab[0] == (N - 1) % 10 && lab[1] == 0);
  CHECK(one[0] == (uint8_t)(N - 1) && one[1] == (uint8_t)(N - 1 + 1024));  // CHW -> HWC
  const int B = 16, S = 3;
  std::vector<uint8_t> img((size_t)S * B * 3072);
  std::vector<int32_t> labs((size_t)S * B);
  CHECK(dtm_loader_start(h, B, S, img.data(), labs.data(), 1, 42) == 0);
  long seen = 0;
  for (int it = 0; it < 40; ++it) {  // consumer reads slots while the worker refills the others
    int s = dtm_loader_next(h);
    for (int b = 0; b < B; ++b) {
      int32_t l = labs[(size_t)s * B + b];
      CHECK(l >= 0 && l < 10);
      seen += img[((size_t)s * B + b) * 3072];
    }
    dtm_loader_release(h, s);
  }
  CHECK(seen > 0);
  dtm_cifar_table_close(h);  // joins the worker while it may be blocked on a full ring
}

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_crc();
  test_tfrecord(dir);
  test_bundle(dir);
  test_cifar_loader(dir);
  std::printf("runtime selftest OK\n");
  return 0;
}
