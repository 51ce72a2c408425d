// Host sanitizer driver for csrc/data/synth_mnist.cpp (the bilinear taps must stay
// inside the bordered source image).  Reads float32 prototypes [classes][4][28][28] from argv[1],
// generates argv[2] samples, writes the uint8 images and int64 labels to argv[3] (raw bytes) so
// the test can compare them with the production library's output.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" int csed_synth_mnist(const float* protos, int classes, int64_t n, uint64_t seed, int train,
                                uint8_t* images, int64_t* labels, int threads);

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  const int classes = 10;
  std::vector<float> protos((size_t)classes * 4 * 784);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(protos.data(), sizeof(float), protos.size(), f) != protos.size()) return 3;
  std::fclose(f);
  const int64_t n = std::atoll(argv[2]);
  std::vector<uint8_t> img((size_t)n * 784);
  std::vector<int64_t> lab((size_t)n);
  if (csed_synth_mnist(protos.data(), classes, n, 7, 1, img.data(), lab.data(), 4) != 0) return 4;
  FILE* o = std::fopen(argv[3], "wb");
  if (!o) return 5;
  std::fwrite(img.data(), 1, img.size(), o);
  std::fwrite(lab.data(), sizeof(int64_t), lab.size(), o);
  std::fclose(o);
  std::printf("synth check ok\n");
  return 0;
}
