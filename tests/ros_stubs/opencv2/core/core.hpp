// stub (syntax check only): the cv::Mat members the map loaders use
#pragma once
#include <cstdint>
namespace cv {
class Mat {
 public:
  int rows = 0, cols = 0;
  template <class T>
  const T* ptr(int) const {
    return nullptr;
  }
};
}  // namespace cv
