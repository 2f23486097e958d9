// stand-in (tests only): the message of dummy_simulator/msg/Belief.msg
// (header; uint8 action; uint8[4] measurement; int32[2] location;
// float32[] belief) as roscpp generates it
#pragma once
#include <array>
#include <cstdint>
#include <vector>

#include <boost/shared_ptr.hpp>
#include <std_msgs/Header.h>

namespace dummy_simulator {
struct Belief {
  std_msgs::Header header;
  uint8_t action = 0;
  std::array<uint8_t, 4> measurement{};
  std::array<int32_t, 2> location{};
  std::vector<float> belief;
};
typedef boost::shared_ptr<Belief> BeliefPtr;
typedef boost::shared_ptr<const Belief> BeliefConstPtr;
}  // namespace dummy_simulator
