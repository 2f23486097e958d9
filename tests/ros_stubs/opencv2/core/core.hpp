// stand-in OpenCV core (tests only): the cv::Mat members the map loaders use
#pragma once
#include <cstdint>
#include <vector>
namespace cv {
class Mat {
 public:
  int rows = 0, cols = 0;
  std::vector<uint8_t> data_;  // 8-bit, one channel, row-major
  template <class T>
  const T* ptr(int y) const {
    return reinterpret_cast<const T*>(data_.data() + (size_t)y * cols);
  }
};
}  // namespace cv
