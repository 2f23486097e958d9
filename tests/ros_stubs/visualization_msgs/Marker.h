// stand-in (tests only): visualization_msgs/Marker fields the MDP node sets
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include <geometry_msgs/Point.h>
#include <std_msgs/ColorRGBA.h>
#include <std_msgs/Header.h>

namespace visualization_msgs {
struct Marker {
  enum : int32_t { SPHERE_LIST = 7 };
  enum : int32_t { ADD = 0 };
  std_msgs::Header header;
  std::string ns;
  int32_t id = 0;
  int32_t type = 0;
  int32_t action = 0;
  geometry_msgs::Pose pose;
  geometry_msgs::Vector3 scale;
  std::vector<geometry_msgs::Point> points;
  std::vector<std_msgs::ColorRGBA> colors;
};
}  // namespace visualization_msgs
