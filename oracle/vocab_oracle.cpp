// vocab_oracle.cpp -- CPU ORACLE for the DBoW2 vocabulary transform
// (Frame::ComputeBoW / KeyFrame::ComputeBoW).  TEST INFRASTRUCTURE ONLY:
// linked into liborb_oracle.so next to orb_oracle.cpp, loaded by tests/ only.
//
// Restates, with the reference's own containers, for DBoW2 as vendored in the
// reference (Thirdparty/DBoW2, TemplatedVocabulary<FORB::TDescriptor, FORB>):
//   * TemplatedVocabulary::loadFromTextFile   TemplatedVocabulary.h:1362-1448
//     (node 0 = root; one node per text line in file order; children in file
//     order; word ids to nodes flagged leaf, in file order)
//   * TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
//                                             TemplatedVocabulary.h:1235-1283
//     (descent: strict '<' so the first child at the minimum distance wins;
//     stops at a node without children, Node::isLeaf :328)
//   * TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
//                                             TemplatedVocabulary.h:1128-1210
//   * BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp:33-90
//   * FeatureVector::addFeature                           FeatureVector.cpp:31-45
//   * FORB::distance (SWAR popcount)                      FORB.cpp:81-101
//   * mustNormalize per scoring type                      ScoringObject.h:53-89
// Called as mpORBvocabulary->transform(desc rows, mBowVec, mFeatVec, 4) from
// src/Frame.cc:439-449 and src/KeyFrame.cc:60-71.
//
// PARITY STATUS: unpinned against a reference binary (OpenCV is absent, so
// DBoW2 cannot be built here, and the ORB vocabulary file ORBvoc.txt is not in
// the reference tree).  Pinned by tests/test_oracle_vocab.py against an
// independent pure-Python restatement on synthetic vocabularies.
// Two reference behaviours have no defined result and are fixed here:
//   * loadFromTextFile's `while(!f.eof())` turns a trailing empty line into a
//     root child with an uninitialised descriptor; this loader skips lines
//     without a parent field.
//   * if the descent hits a leaf above nid_level, the reference leaves the
//     FeatureVector node id uninitialised; here it is the leaf reached.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace vocab_oracle {

typedef uint32_t NodeId;
typedef uint32_t WordId;
typedef double WordValue;

struct Node {  // TemplatedVocabulary::Node, TemplatedVocabulary.h:298-330
  NodeId id = 0;
  WordValue weight = 0;
  std::vector<NodeId> children;
  NodeId parent = 0;
  uint8_t descriptor[32] = {0};
  WordId word_id = 0;
  bool isLeaf() const { return children.empty(); }
};

struct Vocabulary {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  std::vector<Node*> words;
  bool empty() const { return words.empty(); }  // :1009-1012
};

// FORB::distance, FORB.cpp:81-101 (SWAR bit count over 8 int32 words).
static int forb_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; ++i) {
    int32_t pa, pb;
    memcpy(&pa, a + 4 * i, 4);
    memcpy(&pb, b + 4 * i, 4);
    unsigned int v = (unsigned int)(pa ^ pb);
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// Node table as loadFromTextFile builds it (:1400-1444), from the per-line
// fields: parent[i], leaf flag[i], descriptor[i], weight[i] of node i (i >= 1).
static bool build(Vocabulary& V, int k, int L, int scoring, int weighting, int n_nodes,
                  const int32_t* parent, const uint8_t* leaf, const uint8_t* desc,
                  const double* weight) {
  V.k = k; V.L = L; V.scoring = scoring; V.weighting = weighting;
  V.nodes.clear();
  V.words.clear();
  V.nodes.resize(1);
  V.nodes[0].id = 0;
  V.nodes.reserve(n_nodes);
  for (int nid = 1; nid < n_nodes; ++nid) {
    const int pid = parent[nid];
    if (pid < 0 || pid >= nid) return false;
    V.nodes.resize(nid + 1);
    Node& n = V.nodes[nid];
    n.id = nid;
    n.parent = pid;
    V.nodes[pid].children.push_back(nid);
    memcpy(n.descriptor, desc + (size_t)nid * 32, 32);
    n.weight = weight[nid];
    if (leaf[nid]) {
      n.word_id = (WordId)V.words.size();
      V.words.push_back(nullptr);
    }
  }
  for (Node& n : V.nodes)  // pointers taken once the vector stops growing
    if (n.id != 0 && leaf[n.id]) V.words[n.word_id] = &n;
  return true;
}

// transform(feature, word_id, weight, nid, levelsup), :1235-1283.
static void transform_one(const Vocabulary& V, const uint8_t* feature, WordId& word_id,
                          WordValue& weight, NodeId* nid, int levelsup) {
  const int nid_level = V.L - levelsup;
  if (nid_level <= 0 && nid != NULL) *nid = 0;
  NodeId final_id = 0;
  int current_level = 0;
  bool nid_set = nid_level <= 0;
  do {
    ++current_level;
    const std::vector<NodeId>& nodes = V.nodes[final_id].children;
    final_id = nodes[0];
    double best_d = forb_distance(feature, V.nodes[final_id].descriptor);
    for (size_t c = 1; c < nodes.size(); ++c) {
      const NodeId id = nodes[c];
      const double d = forb_distance(feature, V.nodes[id].descriptor);
      if (d < best_d) {
        best_d = d;
        final_id = id;
      }
    }
    if (nid != NULL && current_level == nid_level) {
      *nid = final_id;
      nid_set = true;
    }
  } while (!V.nodes[final_id].isLeaf());
  if (nid != NULL && !nid_set) *nid = final_id;  // reference: uninitialised
  word_id = V.nodes[final_id].word_id;
  weight = V.nodes[final_id].weight;
}

typedef std::map<WordId, WordValue> BowVector;                  // BowVector.h
typedef std::map<NodeId, std::vector<unsigned int>> FeatureVector;  // FeatureVector.h

static void addWeight(BowVector& v, WordId id, WordValue w) {  // BowVector.cpp:33-45
  BowVector::iterator vit = v.lower_bound(id);
  if (vit != v.end() && !(v.key_comp()(id, vit->first))) vit->second += w;
  else v.insert(vit, BowVector::value_type(id, w));
}

static void addIfNotExist(BowVector& v, WordId id, WordValue w) {  // :48-56
  BowVector::iterator vit = v.lower_bound(id);
  if (vit == v.end() || (v.key_comp()(id, vit->first))) v.insert(vit, BowVector::value_type(id, w));
}

static void normalize(BowVector& v, int l2) {  // :59-81
  double norm = 0.0;
  if (!l2) {
    for (auto& it : v) norm += fabs(it.second);
  } else {
    for (auto& it : v) norm += it.second * it.second;
    norm = sqrt(norm);
  }
  if (norm > 0.0)
    for (auto& it : v) it.second /= norm;
}

static void addFeature(FeatureVector& fv, NodeId id, unsigned int i) {  // FeatureVector.cpp:31-45
  FeatureVector::iterator vit = fv.lower_bound(id);
  if (vit != fv.end() && vit->first == id) {
    vit->second.push_back(i);
  } else {
    vit = fv.insert(vit, FeatureVector::value_type(id, std::vector<unsigned int>()));
    vit->second.push_back(i);
  }
}

// ScoringObject.h:74-89: every scoring but DOT_PRODUCT (5) normalises, with
// L2 for L2_NORM (1) and L1 otherwise.
static bool must_normalize(int scoring, int& l2) {
  l2 = scoring == 1;
  return scoring != 5;
}

// transform(features, v, fv, levelsup), :1128-1210.
static void transform(const Vocabulary& V, int n, const uint8_t* desc, int levelsup,
                      BowVector& v, FeatureVector& fv, WordId* fword, NodeId* fnode) {
  v.clear();
  fv.clear();
  if (V.empty()) return;
  int l2 = 0;
  const bool must = must_normalize(V.scoring, l2);
  const bool tf = V.weighting == 0 /*TF_IDF*/ || V.weighting == 1 /*TF*/;
  for (int i = 0; i < n; ++i) {
    WordId id;
    NodeId nid = 0;
    WordValue w;
    transform_one(V, desc + (size_t)i * 32, id, w, &nid, levelsup);
    if (fword) fword[i] = w > 0 ? id : 0xFFFFFFFFu;
    if (fnode) fnode[i] = nid;
    if (w > 0) {
      if (tf) addWeight(v, id, w);
      else addIfNotExist(v, id, w);
      addFeature(fv, nid, (unsigned int)i);
    }
  }
  if (tf && !v.empty() && !must) {
    const double nd = v.size();
    for (auto& it : v) it.second /= nd;
  }
  if (must) normalize(v, l2);
}

// loadFromTextFile, :1362-1448: header "k L scoring weighting", then per node
// "parent isLeaf d0 .. d31 weight".
static bool load_text(const char* path, Vocabulary& V, std::vector<int32_t>& parent,
                      std::vector<uint8_t>& leaf, std::vector<uint8_t>& desc,
                      std::vector<double>& weight) {
  std::ifstream f(path);
  if (!f.is_open() || f.eof()) return false;
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int k = -1, L = -1, n1 = -1, n2 = -1;
  ss >> k >> L >> n1 >> n2;
  if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return false;
  parent.assign(1, 0);
  leaf.assign(1, 0);
  desc.assign(32, 0);
  weight.assign(1, 0.0);
  while (!f.eof()) {
    std::string snode;
    std::getline(f, snode);
    std::stringstream ssnode;
    ssnode << snode;
    int pid;
    if (!(ssnode >> pid)) continue;  // trailing empty line (see header)
    int nIsLeaf = 0;
    ssnode >> nIsLeaf;
    uint8_t d[32] = {0};
    for (int i = 0; i < 32; ++i) {  // FORB::fromString, FORB.cpp:120-135
      int v;
      ssnode >> v;
      if (!ssnode.fail()) d[i] = (unsigned char)v;
    }
    double w = 0;
    ssnode >> w;
    parent.push_back(pid);
    leaf.push_back(nIsLeaf > 0);
    desc.insert(desc.end(), d, d + 32);
    weight.push_back(w);
  }
  return build(V, k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(),
               weight.data());
}

}  // namespace vocab_oracle

using namespace vocab_oracle;

extern "C" {

// Flattened outputs: BowVector as (words ascending, values); FeatureVector as
// CSR (node ids ascending, offsets[n_fv + 1], feature indices).  Per-feature
// word id (0xFFFFFFFF = stopped, weight <= 0) and FeatureVector node id.
// Returns 0, or -1 for a malformed node table.
int oracle_vocab_transform(int k, int L, int scoring, int weighting, int n_nodes,
                           const int32_t* parent, const uint8_t* leaf, const uint8_t* node_desc,
                           const double* node_weight, int n, const uint8_t* desc, int levelsup,
                           uint32_t* bow_words, double* bow_values, int* n_words,
                           uint32_t* fv_nodes, int32_t* fv_offs, uint32_t* fv_feats, int* n_fv,
                           uint32_t* feat_word, uint32_t* feat_node) {
  Vocabulary V;
  if (!build(V, k, L, scoring, weighting, n_nodes, parent, leaf, node_desc, node_weight))
    return -1;
  BowVector v;
  FeatureVector fv;
  transform(V, n, desc, levelsup, v, fv, feat_word, feat_node);
  int i = 0;
  for (auto& it : v) {
    bow_words[i] = it.first;
    bow_values[i] = it.second;
    ++i;
  }
  *n_words = i;
  int j = 0, o = 0;
  fv_offs[0] = 0;
  for (auto& it : fv) {
    fv_nodes[j] = it.first;
    for (unsigned int f : it.second) fv_feats[o++] = f;
    fv_offs[++j] = o;
  }
  *n_fv = j;
  return 0;
}

// Parses a vocabulary text file the way loadFromTextFile does.  Writes the
// header (k, L, scoring, weighting) and, when cap >= the node count, the node
// table; returns the node count (including the root), or -1.
int oracle_vocab_parse_text(const char* path, int32_t* header, int cap, int32_t* parent,
                            uint8_t* leaf, uint8_t* desc, double* weight) {
  Vocabulary V;
  std::vector<int32_t> p;
  std::vector<uint8_t> l, d;
  std::vector<double> w;
  if (!load_text(path, V, p, l, d, w)) return -1;
  header[0] = V.k; header[1] = V.L; header[2] = V.scoring; header[3] = V.weighting;
  const int n = (int)p.size();
  if (cap >= n) {
    memcpy(parent, p.data(), n * 4);
    memcpy(leaf, l.data(), n);
    memcpy(desc, d.data(), (size_t)n * 32);
    memcpy(weight, w.data(), (size_t)n * 8);
  }
  return n;
}

// CPU baseline for the transform (bench leg): builds the tree once, then
// runs transform() over n_frames frames of n_per_frame descriptors each on
// this thread; returns the seconds spent in transform() only (the reference
// loads the vocabulary once at start-up, System::System src/System.cc).
double oracle_vocab_time(int k, int L, int scoring, int weighting, int n_nodes,
                         const int32_t* parent, const uint8_t* leaf, const uint8_t* node_desc,
                         const double* node_weight, int n_frames, int n_per_frame,
                         const uint8_t* desc, int levelsup) {
  Vocabulary V;
  if (!build(V, k, L, scoring, weighting, n_nodes, parent, leaf, node_desc, node_weight))
    return -1.0;
  BowVector v;
  FeatureVector fv;
  const auto t0 = std::chrono::steady_clock::now();
  for (int f = 0; f < n_frames; ++f)
    transform(V, n_per_frame, desc + (size_t)f * n_per_frame * 32, levelsup, v, fv, nullptr,
              nullptr);
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
