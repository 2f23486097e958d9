// Drives one planner node adapter (ros/src/{pomdp,mdp}/path_planning_2d_pp2.cpp)
// through the stand-in roscpp transport of ros/ros.h, the way the reference's
// node mains and the dummy simulator drive the nodes
// (src/{pomdp,mdp}/path_planning_2d_node.cpp: construct with the private
// NodeHandle, initialize(), then one beliefCallback per ~belief message).
// Built with -DPP2_NODE_POMDP or -DPP2_NODE_MDP by tests/test_gpu_ros_nodes.py
// and linked against libpp2_hip.so.
//
//   run_node <params> <messages> <out> [save]
//   params:   lines "name value" (the launch-file parameters)
//   messages: int32 count, int32 kind, int32 n; then per message uint8
//             action, uint8 measurement[4] and either n floats (kind 0: the
//             belief) or an int32 cell (kind 1: a one-hot belief of n cells)
//   out:      the published ~control bytes, one per line; then for the MDP
//             node "markers <optimal_cost count> <optimal_action count>
//             <points per marker>"; with "save", the ~save_data service is
//             called after the last message ("save_data <0|1>").
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <dummy_simulator/Belief.h>
#include <std_msgs/Byte.h>
#include <std_srvs/Trigger.h>
#include <visualization_msgs/Marker.h>

#ifdef PP2_NODE_POMDP
#include <path_planning_2d/pomdp_path_planning_2d.h>
typedef path_planning_2d::PomdpPathPlanning2d Node;
#else
#include <path_planning_2d/mdp_path_planning_2d.h>
typedef path_planning_2d::MdpPathPlanning2d Node;
#endif

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: run_node <params> <messages> <out> [save]\n");
    return 2;
  }
  {
    std::ifstream pf(argv[1]);
    std::string line;
    while (std::getline(pf, line)) {
      std::istringstream ls(line);
      std::string k, v;
      if (ls >> k >> v) ros::stub::params()[k] = v;
    }
  }
  ros::init(argc, argv, "path_planner");
  ros::NodeHandle nh("~");
  Node::Ptr node(new Node(nh));
  if (!node->initialize()) {
    std::fprintf(stderr, "initialize() failed\n");
    return 3;
  }
  FILE* mf = std::fopen(argv[2], "rb");
  if (!mf) return 4;
  int32_t hdr[3];
  if (std::fread(hdr, sizeof hdr, 1, mf) != 1) return 4;
  const int count = hdr[0], kind = hdr[1], n = hdr[2];
  auto& sub = ros::stub::subscribers<dummy_simulator::Belief>();
  if (!sub.count("belief")) return 5;
  for (int i = 0; i < count; ++i) {
    dummy_simulator::BeliefPtr msg(new dummy_simulator::Belief);
    if (std::fread(&msg->action, 1, 1, mf) != 1 ||
        std::fread(msg->measurement.data(), 1, 4, mf) != 4)
      return 4;
    msg->belief.assign((size_t)n, 0.0f);
    if (kind == 0) {
      if (std::fread(msg->belief.data(), sizeof(float), (size_t)n, mf) != (size_t)n) return 4;
    } else {
      int32_t cell = 0;
      if (std::fread(&cell, sizeof cell, 1, mf) != 1 || cell < 0 || cell >= n) return 4;
      msg->belief[(size_t)cell] = 1.0f;
    }
    sub["belief"](msg);
  }
  std::fclose(mf);
  FILE* of = std::fopen(argv[3], "w");
  if (!of) return 6;
  for (const std_msgs::Byte& b : ros::stub::published<std_msgs::Byte>()["control"])
    std::fprintf(of, "%d\n", (int)b.data);
  auto& mk = ros::stub::published<visualization_msgs::Marker>();
  if (mk.count("optimal_cost"))
    std::fprintf(of, "markers %zu %zu %zu\n", mk["optimal_cost"].size(),
                 mk["optimal_action"].size(),
                 mk["optimal_cost"].empty() ? (size_t)0 : mk["optimal_cost"][0].points.size());
  if (argc > 4 && std::string(argv[4]) == "save") {
    auto& srv = ros::stub::services<std_srvs::Trigger::Request, std_srvs::Trigger::Response>();
    std_srvs::Trigger::Request q;
    std_srvs::Trigger::Response r;
    const bool called = srv.count("save_data") && srv["save_data"](q, r);
    std::fprintf(of, "save_data %d\n", called && r.success ? 1 : 0);
  }
  std::fclose(of);
  return 0;
}
