// stand-in (tests only): the interface of the catkin package's unchanged
// base class, include/path_planning_2d/path_planning_2d_base.h:31-93 of the
// reference -- the pure virtuals the node classes override and the protected
// members they use.  Like the reference's, the destructor is NOT virtual
// (:43); the node mains hold the derived classes' own Ptr types.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>

#include <boost/shared_ptr.hpp>
#include <dummy_simulator/Belief.h>
#include <ros/ros.h>

namespace path_planning_2d {

class PathPlanning2dBase {
 public:
  typedef boost::shared_ptr<PathPlanning2dBase> Ptr;
  typedef boost::shared_ptr<const PathPlanning2dBase> ConstPtr;
  explicit PathPlanning2dBase(ros::NodeHandle& n) : nh(n) {}
  PathPlanning2dBase(const PathPlanning2dBase&) = delete;
  ~PathPlanning2dBase() {}
  virtual bool initialize() = 0;

 protected:
  virtual bool loadParameters() = 0;
  virtual bool createRosIO() = 0;
  virtual void beliefCallback(const dummy_simulator::BeliefConstPtr& belief) = 0;
  virtual void loadMapFromFile() = 0;

  std::string map_path;
  uint32_t map_width = 0, map_height = 0;
  double map_resolution = 0.0;
  uint8_t* grid_map = nullptr;
  int32_t goal[2] = {0, 0};
  float discount_factor = 0.0f;
  ros::NodeHandle nh;
  std::string fixed_frame_id, robot_frame_id;
  ros::Publisher control_pub;
  ros::Subscriber belief_sub;
  FILE* planning_time_fid = nullptr;
};

}  // namespace path_planning_2d
