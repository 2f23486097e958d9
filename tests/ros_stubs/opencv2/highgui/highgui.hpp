// stand-in OpenCV highgui (tests only): cv::imread of an 8-bit greyscale
// binary PGM (P5), which is what tests/test_gpu_ros_nodes.py writes for the
// reference's map PNGs (their pixels are 0 or 255); an empty Mat otherwise.
#pragma once
#include <cstdio>
#include <string>
#include <opencv2/core/core.hpp>
namespace cv {
enum { IMREAD_GRAYSCALE = 0 };
inline Mat imread(const std::string& path, int) {
  Mat m;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return m;
  int w = 0, h = 0, maxv = 0;
  if (std::fscanf(f, "P5 %d %d %d", &w, &h, &maxv) == 3 && maxv == 255 && std::fgetc(f) != EOF) {
    m.data_.resize((size_t)w * h);
    if (std::fread(m.data_.data(), 1, m.data_.size(), f) == m.data_.size()) {
      m.rows = h;
      m.cols = w;
    } else {
      m.data_.clear();
    }
  }
  std::fclose(f);
  return m;
}
}  // namespace cv
