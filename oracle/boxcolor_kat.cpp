// boxcolor_kat.cpp -- TEST INFRASTRUCTURE (oracle pinning), never shipped or linked by the product.
//
// BoundingBox::setRandomColor (src/BoundingBox.cpp:163-165) builds the colour as
//   Eigen::Vector3f(rand() / (float)RAND_MAX, rand() / (float)RAND_MAX, rand() / (float)RAND_MAX)
// C++ leaves the evaluation order of those three arguments unspecified. This generator
// evaluates that constructor expression as the reference's build would -- this image's g++, the
// reference's vendored Eigen, glibc rand() in a fresh process (seed 1) -- for the first 4,480 boxes
// (the 1M soup's box count) and writes the colours to tests/golden/boxcolor_kat.bin, which pins
// rt_box_colors_random and the oracle. (g++ on x86-64 evaluates the arguments right to left: the
// first rand() call lands in the blue channel.)
//
// Build: oracle/Makefile target boxcolor_kat (only where /root/reference exists).
#include <Eigen/Dense>

#include <cstdio>
#include <cstdlib>

static Eigen::Vector3f set_random_color() {  // the expression of BoundingBox.cpp:164
  return Eigen::Vector3f(rand() / (float)RAND_MAX, rand() / (float)RAND_MAX, rand() / (float)RAND_MAX);
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "boxcolor_kat.bin";
  const int n = 4480;
  FILE* f = std::fopen(path, "wb");
  if (!f) { std::perror(path); return 1; }
  for (int b = 0; b < n; b++) {
    const Eigen::Vector3f c = set_random_color();
    std::fwrite(c.data(), 4, 3, f);
  }
  std::fclose(f);
  std::printf("wrote %d box colours to %s\n", n, path);
  return 0;
}
