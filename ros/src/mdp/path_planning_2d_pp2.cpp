// MdpPathPlanning2d on libpp2_hip.so: replaces src/mdp/path_planning_2d.cu of
// the reference (class body :59-487) in the catkin package.  Header
// (include/path_planning_2d/mdp_path_planning_2d.h), node main, launch files,
// parameters and topics are unchanged.  The model and value iteration run in
// one pp2_ctx; valueIteration keeps the reference's stopping rule (blocks of
// 100 sweeps until the inf-norm of the change is <= 1e-3 * 5 / (1 - gamma),
// :207-269) without its OpenCV windows, then the optimal cost and action are
// downloaded once for the table-lookup beliefCallback.
//
// Syntax-checked here (tests/test_ros_adapters.py, stand-in ROS / OpenCV
// headers in tests/ros_stubs/); no ROS / OpenCV in the image to link it.
#include <cstdio>
#include <cstdlib>

#include <opencv2/core/core.hpp>
#include <opencv2/highgui/highgui.hpp>

#include <std_msgs/Byte.h>
#include <visualization_msgs/Marker.h>

#include <pp2.h>

#include <path_planning_2d/mdp_path_planning_2d.h>

namespace path_planning_2d {

namespace {

pp2_ctx* g_ctx = nullptr;  // the node's grid on the GPU (one node per process)

bool pp2_ok(int status, const char* what) {
  if (status == PP2_OK) return true;
  ROS_ERROR("%s failed (%s): %s", what, pp2_status_string(status), pp2_last_error());
  return false;
}

// RViz colour of each action (publishSolution's palette: 0 black, 1 blue,
// 2 green, 3 cyan, 4 white, 5 red, 6 magenta, 7 yellow, 8 white).
constexpr float kActionRGB[9][3] = {{0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {0, 1, 1}, {1, 1, 1},
                                    {1, 0, 0}, {1, 0, 1}, {1, 1, 0}, {1, 1, 1}};

visualization_msgs::Marker grid_marker(const std::string& frame, int id, double res) {
  visualization_msgs::Marker m;
  m.header.stamp = ros::Time::now();
  m.header.frame_id = frame;
  m.ns = "MDP solution";
  m.id = id;
  m.type = visualization_msgs::Marker::SPHERE_LIST;
  m.action = visualization_msgs::Marker::ADD;
  m.pose.orientation.w = 1.0;
  m.scale.x = m.scale.y = m.scale.z = res;
  return m;
}

}  // namespace

MdpPathPlanning2d::MdpPathPlanning2d(ros::NodeHandle& n) : PathPlanning2dBase(n) {}

MdpPathPlanning2d::~MdpPathPlanning2d() {
  if (g_ctx) pp2_destroy(g_ctx);
  g_ctx = nullptr;
  free(grid_map);
  free(optimal_cost);
  free(optimal_action);
}

bool MdpPathPlanning2d::loadParameters() {
  const bool ok = nh.getParam("map_path", map_path) && nh.getParam("goal_x", goal[0]) &&
                  nh.getParam("goal_y", goal[1]) &&
                  nh.getParam("discount_factor", discount_factor) &&
                  nh.getParam("map_resolution", map_resolution);
  nh.param<std::string>("fixed_frame_id", fixed_frame_id, "map");
  nh.param<std::string>("robot_frame_id", robot_frame_id, "robot");
  return ok;
}

// 1 where the grey level is <= 250 (the reference's THRESH_BINARY_INV at 250).
void MdpPathPlanning2d::loadMapFromFile() {
  const cv::Mat img = cv::imread(map_path, cv::IMREAD_GRAYSCALE);
  map_height = img.rows;
  map_width = img.cols;
  grid_map = static_cast<uint8_t*>(malloc((size_t)map_height * map_width));
  for (uint32_t y = 0; y < map_height; ++y) {
    const uint8_t* row = img.ptr<uint8_t>(y);
    for (uint32_t x = 0; x < map_width; ++x) grid_map[(size_t)y * map_width + x] = row[x] <= 250;
  }
}

bool MdpPathPlanning2d::initialize() {
  if (!loadParameters()) {
    ROS_WARN("Cannot load all required parameters...");
    return false;
  }
  loadMapFromFile();
  if (grid_map[(size_t)goal[1] * map_width + goal[0]]) {
    ROS_ERROR("The assigned goal (%d %d) is at a occupied cell...", goal[0], goal[1]);
    return false;
  }
  if (!pp2_ok(pp2_create(&g_ctx, /*device=*/0, map_height, map_width, grid_map, goal[0],
                         goal[1], discount_factor),
              "pp2_create") ||
      !pp2_ok(pp2_model_generate(g_ctx), "model generation"))
    return false;
  std::printf("Solve MDP with value iteration...\n");
  valueIteration();
  const size_t hw = (size_t)map_height * map_width;
  optimal_cost = static_cast<float*>(malloc(hw * sizeof(float)));
  optimal_action = static_cast<uint8_t*>(malloc(hw));
  if (!pp2_ok(pp2_mdp_get(g_ctx, optimal_cost, optimal_action), "downloading the solution"))
    return false;
  if (!createRosIO()) {
    ROS_WARN("Cannot load all ROS I/O...");
    return false;
  }
  publishSolution();
  std::printf("Initialization finished...\n");
  return true;
}

void MdpPathPlanning2d::valueIteration() {
  int sweeps = 0;
  double inf_norm = 0.0;
  const ros::Time t0 = ros::Time::now();
  if (pp2_ok(pp2_mdp_solve(g_ctx, /*max_sweeps=*/0, &sweeps, &inf_norm), "value iteration"))
    std::printf("value iteration: %d sweeps, inf-norm %f, %f s\n", sweeps, inf_norm,
                (ros::Time::now() - t0).toSec());
}

// The reference's policyIteration drives the dead cudaOneStepPolicyEvaluation /
// cudaPolicyImprovment kernels and is never called (initialize keeps it
// commented out); value iteration reaches the same fixed point.
void MdpPathPlanning2d::policyIteration() { valueIteration(); }

bool MdpPathPlanning2d::createRosIO() {
  control_pub = nh.advertise<std_msgs::Byte>("control", 1);
  optimal_cost_pub = nh.advertise<visualization_msgs::Marker>("optimal_cost", 1, true);
  optimal_action_pub = nh.advertise<visualization_msgs::Marker>("optimal_action", 1, true);
  belief_sub = nh.subscribe("belief", 1, &MdpPathPlanning2d::beliefCallback, this);
  return true;
}

// The action of the belief's mode (first maximum above 0; cell 0 otherwise).
void MdpPathPlanning2d::beliefCallback(const dummy_simulator::BeliefConstPtr& msg) {
  float best = 0.0f;
  size_t mode = 0;
  for (size_t i = 0; i < msg->belief.size(); ++i)
    if (msg->belief[i] > best) best = msg->belief[mode = i];
  std_msgs::Byte out;
  out.data = optimal_action[mode];
  control_pub.publish(out);
}

void MdpPathPlanning2d::publishSolution() {
  const double max_cost = 5.0 / (1.0 - discount_factor);
  visualization_msgs::Marker cost = grid_marker(fixed_frame_id, 0, map_resolution);
  visualization_msgs::Marker act = grid_marker(fixed_frame_id, 1, map_resolution);
  const size_t hw = (size_t)map_height * map_width;
  cost.points.resize(hw);
  cost.colors.resize(hw);
  act.points.resize(hw);
  act.colors.resize(hw);
  for (size_t i = 0; i < hw; ++i) {
    const double px = map_resolution * (i % map_width + 0.5);
    const double py = map_resolution * (i / map_width + 0.5);
    cost.points[i].x = act.points[i].x = px;
    cost.points[i].y = act.points[i].y = py;
    const float shade = (float)(1.0 - optimal_cost[i] / max_cost);
    cost.colors[i].r = cost.colors[i].g = cost.colors[i].b = shade;
    cost.colors[i].a = 1.0f;
    const float* rgb = kActionRGB[optimal_action[i] < 9 ? optimal_action[i] : 0];
    act.colors[i].r = rgb[0];
    act.colors[i].g = rgb[1];
    act.colors[i].b = rgb[2];
    act.colors[i].a = 1.0f;
  }
  optimal_cost_pub.publish(cost);
  optimal_action_pub.publish(act);
}

}  // namespace path_planning_2d
