// stand-in (tests only)
#pragma once
namespace geometry_msgs {
struct Point {
  double x = 0, y = 0, z = 0;
};
struct Quaternion {
  double x = 0, y = 0, z = 0, w = 0;
};
struct Vector3 {
  double x = 0, y = 0, z = 0;
};
struct Pose {
  Point position;
  Quaternion orientation;
};
}  // namespace geometry_msgs
