// stand-in (tests only): the interface of the catkin package's unchanged
// MDP node class, include/path_planning_2d/mdp_path_planning_2d.h:24-78 of
// the reference -- the members ros/src/mdp/path_planning_2d_pp2.cpp defines.
#pragma once
#include <cstdint>

#include "path_planning_2d_base.h"

namespace path_planning_2d {

class MdpPathPlanning2d : public PathPlanning2dBase {
 public:
  typedef boost::shared_ptr<MdpPathPlanning2d> Ptr;
  explicit MdpPathPlanning2d(ros::NodeHandle& n);
  ~MdpPathPlanning2d();
  virtual bool initialize();

 private:
  virtual bool loadParameters();
  virtual bool createRosIO();
  virtual void beliefCallback(const dummy_simulator::BeliefConstPtr& belief);
  virtual void loadMapFromFile();
  void publishSolution();
  void valueIteration();
  void policyIteration();

  float* optimal_cost = nullptr;
  uint8_t* optimal_action = nullptr;
  ros::Publisher optimal_cost_pub;
  ros::Publisher optimal_action_pub;
};

}  // namespace path_planning_2d
