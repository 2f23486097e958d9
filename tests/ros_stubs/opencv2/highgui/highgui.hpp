// stub (syntax check only): cv::imread
#pragma once
#include <string>
#include <opencv2/core/core.hpp>
namespace cv {
enum { IMREAD_GRAYSCALE = 0 };
inline Mat imread(const std::string&, int) { return Mat(); }
}  // namespace cv
