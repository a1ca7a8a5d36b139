// Host-side tables of the device annotation serialiser (ksched_json.h):
// every string piece ksg_annotate writes, escaped once by the annotator
// (ksched_annotate.cpp) and packed into flat arrays for the upload.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "ksched.h"

struct JsonHostTables {
  std::string node_keys;                 // "<name>": per node, node index order
  std::vector<int64_t> node_key_off;     // [N + 1]
  std::vector<int32_t> node_order;       // [N] node indices sorted bytewise by name
  std::string plugin_keys;               // "<name>": per plugin id
  std::vector<int32_t> plugin_key_off;   // [KSG_NPLUGINS + 1]
  int32_t by_name[KSG_NPLUGINS];         // plugin ids sorted by name
  std::string msgs;                      // quoted messages, index pl * 8 + reason (empty: none)
  std::vector<int32_t> msg_off;          // [KSG_NPLUGINS * 8 + 1]
  std::string taint_msgs;                // quoted "node(s) had untolerated taint {k: v}" per vocab id
  std::vector<int32_t> taint_msg_off;    // [V + 1]
  std::string fit_parts;                 // unquoted "Too many pods", "Insufficient <res r>" ...
  std::vector<int32_t> fit_part_off;     // [1 + R + 1]
  int32_t n_res = 0, n_taint_vocab = 0, max_taints = 0;
};

// ksched_annotate.cpp
int ksg_annotator_json_tables(const ksg_annotator* a, JsonHostTables* out);
