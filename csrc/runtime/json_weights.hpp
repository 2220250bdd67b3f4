// Native reader/writer for the reference's per-neuron JSON weight format.
//
// Formats:
//   model config  {"layers":[{"type","nodes","neurons":[{"weights":[in],"bias","activation"}]}],
//                  "layer_distribution":[...]}                 (/root/reference/config/config_sample.json)
//   notebook form {"model":{"layers":[...]}, "inference_metrics":{...}}
//                  (/root/reference/scripts/Centralized_MNIST_Experimentation.ipynb:493-506)
//   stage file    {"layer_1":[neurons...], "layer_2":[...]}
//                  (/root/reference/src/run_grpc_fcnn.py:108-127, read by src/grpc_node.py:43-55)
// One JSON neuron = one OUTPUT unit whose `weights` has length in_dim, i.e. a row of an
// nn.Linear weight [out][in] (/root/reference/src/grpc_node.py:51 uses the transpose).
//
// A 784-8192-8192-10 model is >1 GB of JSON text; Python's json builds ~10^8 float objects
// for it. This parser is schema-directed and streaming: numbers go straight into float32
// row-major buffers, unknown keys are skipped without materialising anything.
#pragma once
#include <string>
#include <vector>

namespace dnn {

struct ParsedLayer {
  std::string key;   // "layer_k" for stage files, "" otherwise
  std::string type;  // "hidden"/"output" (may be empty)
  int nodes = 0;     // declared "nodes" (or number of neurons when absent)
  int in_dim = 0;
  std::string activation = "linear";  // activation of the FIRST neuron (grpc_node.py:53)
  bool mixed_activation = false;      // some neuron disagrees with the first one
  std::vector<float> weights;         // [num_neurons][in_dim]
  std::vector<float> bias;            // [num_neurons]
};

struct ParsedModel {
  std::vector<ParsedLayer> layers;
  std::vector<int> layer_distribution;
  bool has_distribution = false;
  bool wrapped = false;     // {"model":{...}} notebook form
  bool stage_file = false;  // {"layer_k": [...]} form (sorted by integer k)
};

ParsedModel parse_neuron_json_file(const std::string& path);
ParsedModel parse_neuron_json(const char* data, size_t size);

struct LayerOut {
  int out = 0, in = 0;
  const float* w = nullptr;  // [out][in]
  const float* b = nullptr;  // [out]
  std::string activation, type;
};

// stage_file=false: {"layers":[...], "layer_distribution":[...]}; true: {"layer_1":[...],...}
void write_neuron_json_file(const std::string& path, const std::vector<LayerOut>& layers,
                            const std::vector<int>& distribution, bool stage_file);

// Inputs file {"examples":[{"input":[...], "label":int}, ...]} or the raw-list form
// {"examples":[[...], ...]} (/root/reference/scripts/manual_nn.py:85, run_grpc_inference.py:187).
// Nested (2-D) inputs are flattened row-major; `outer_len` keeps len(input) of the first example,
// which is what the reference partitioner uses as the input dimension
// (/root/reference/src/run_grpc_fcnn.py:190-192).
struct ParsedExamples {
  std::vector<float> x;     // [n][dim]
  std::vector<int> labels;  // [n], -1 when absent
  int n = 0, dim = 0, outer_len = 0;
  bool raw_list = false;
};
ParsedExamples parse_examples_json_file(const std::string& path);
ParsedExamples parse_examples_json(const char* data, size_t size);

}  // namespace dnn
