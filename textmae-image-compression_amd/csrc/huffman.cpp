// Huffman side information of the Kodak eval harness: HuffmanCoding (reference utils/huffman.py:6-171)
// codes the decoder's unshuffle indices (ids_restore, testing.py:71-74) into a string of '0'/'1'
// characters whose length is the side-info bit count in the bpp (testing.py:88-89).
//
// Host C++ (tree building is sequential; the input is B x L <= a few thousand indices).  Bit-for-bit the
// same code table as the reference, which depends on Python's heapq and dict semantics:
//   * symbols are counted in first-occurrence order (defaultdict insertion order, huffman.py:55-59) and
//     pushed onto the heap in that order (60-62);
//   * the heap is CPython's heapq (heappush = append + _siftdown; heappop = pop last, move it to the root,
//     _siftup then _siftdown) ordered by Node.__lt__ = freq only (huffman.py:30-40), so equal frequencies
//     resolve by heap position exactly as in the reference;
//   * build_tree pops two nodes, merges them as (left = first popped, right = second), pushes (68-78);
//   * codes come from a pre-order walk, left '0', right '1' (80-103); a lone symbol gets the empty code.
#include <stdint.h>
#include <string.h>

#include <unordered_map>
#include <vector>

#include "../../include/tmae.h"

void tmae_set_error(int code, const char* fmt, ...);

namespace {

struct Node {
  int64_t value;
  bool leaf;
  int64_t freq;
  int left, right;  // node indices, -1 for none
};

struct Heap {
  std::vector<Node>& nodes;
  std::vector<int> h;
  bool lt(int a, int b) const { return nodes[a].freq < nodes[b].freq; }
  // heapq._siftdown(heap, startpos, pos)
  void siftdown(size_t start, size_t pos) {
    const int item = h[pos];
    while (pos > start) {
      const size_t parent = (pos - 1) >> 1;
      if (lt(item, h[parent])) {
        h[pos] = h[parent];
        pos = parent;
        continue;
      }
      break;
    }
    h[pos] = item;
  }
  // heapq._siftup(heap, pos)
  void siftup(size_t pos) {
    const size_t end = h.size(), start = pos;
    const int item = h[pos];
    size_t child = 2 * pos + 1;
    while (child < end) {
      const size_t right = child + 1;
      if (right < end && !lt(h[child], h[right])) child = right;
      h[pos] = h[child];
      pos = child;
      child = 2 * pos + 1;
    }
    h[pos] = item;
    siftdown(start, pos);
  }
  void push(int n) {
    h.push_back(n);
    siftdown(0, h.size() - 1);
  }
  int pop() {
    const int last = h.back();
    h.pop_back();
    if (h.empty()) return last;
    const int ret = h[0];
    h[0] = last;
    siftup(0);
    return ret;
  }
};

struct Table {
  std::vector<int64_t> sym;
  std::vector<int32_t> len;
  std::vector<uint64_t> code;  // MSB-first bits in the low `len` bits
};

void walk(const std::vector<Node>& nodes, int n, uint64_t code, int len, Table& t) {
  if (n < 0) return;
  if (nodes[n].leaf) {
    t.sym.push_back(nodes[n].value);
    t.len.push_back(len);
    t.code.push_back(code);
  }
  walk(nodes, nodes[n].left, code << 1, len + 1, t);
  walk(nodes, nodes[n].right, (code << 1) | 1u, len + 1, t);
}

}  // namespace

extern "C" int tmae_huffman_build(const int64_t* values, long long n, int64_t* syms, int32_t* lens, uint64_t* codes,
                                  int cap, int* nsym) {
  if (!values || n <= 0 || !syms || !lens || !codes || !nsym) {
    tmae_set_error(TMAE_EINVAL, "tmae_huffman_build: bad arguments");
    return TMAE_EINVAL;
  }
  std::vector<Node> nodes;
  std::unordered_map<int64_t, int> where;
  where.reserve((size_t)n * 2);
  for (long long i = 0; i < n; ++i) {
    auto it = where.find(values[i]);
    if (it == where.end()) {
      where.emplace(values[i], (int)nodes.size());
      nodes.push_back(Node{values[i], true, 1, -1, -1});
    } else {
      nodes[it->second].freq += 1;
    }
  }
  const int nleaf = (int)nodes.size();
  if (nleaf > cap) {
    tmae_set_error(TMAE_EINVAL, "tmae_huffman_build: %d distinct values exceed the table capacity %d", nleaf, cap);
    return TMAE_EINVAL;
  }
  nodes.reserve(2 * nleaf);
  Heap heap{nodes, {}};
  for (int i = 0; i < nleaf; ++i) heap.push(i);
  while (heap.h.size() > 1) {
    const int a = heap.pop();
    const int b = heap.pop();
    nodes.push_back(Node{0, false, nodes[a].freq + nodes[b].freq, a, b});
    heap.push((int)nodes.size() - 1);
  }
  Table t;
  walk(nodes, heap.pop(), 0, 0, t);
  for (size_t i = 0; i < t.sym.size(); ++i) {
    if (t.len[i] > 64) {
      tmae_set_error(TMAE_EINVAL, "tmae_huffman_build: code longer than 64 bits");
      return TMAE_EINVAL;
    }
    syms[i] = t.sym[i];
    lens[i] = t.len[i];
    codes[i] = t.code[i];
  }
  *nsym = (int)t.sym.size();
  return TMAE_OK;
}

// HuffmanCoding.encode (huffman.py:105-119): '0'/'1' characters; *nbits = length (out may be NULL to size)
extern "C" int tmae_huffman_encode(const int64_t* values, long long n, const int64_t* syms, const int32_t* lens,
                                   const uint64_t* codes, int nsym, char* out, long long cap, long long* nbits) {
  if (!values || !syms || !lens || !codes || !nbits || nsym <= 0) {
    tmae_set_error(TMAE_EINVAL, "tmae_huffman_encode: bad arguments");
    return TMAE_EINVAL;
  }
  std::unordered_map<int64_t, int> idx;
  idx.reserve((size_t)nsym * 2);
  for (int i = 0; i < nsym; ++i) idx.emplace(syms[i], i);
  long long pos = 0;
  for (long long i = 0; i < n; ++i) {
    auto it = idx.find(values[i]);
    if (it == idx.end()) {
      tmae_set_error(TMAE_EINVAL, "tmae_huffman_encode: value %lld has no code (KeyError in the reference)",
                     (long long)values[i]);
      return TMAE_EINVAL;
    }
    const int k = it->second, L = lens[k];
    if (out) {
      if (pos + L > cap) {
        tmae_set_error(TMAE_EINVAL, "tmae_huffman_encode: output buffer too small");
        return TMAE_EINVAL;
      }
      for (int b = L - 1; b >= 0; --b) out[pos++] = ((codes[k] >> b) & 1u) ? '1' : '0';
    } else {
      pos += L;
    }
  }
  *nbits = pos;
  return TMAE_OK;
}

// HuffmanCoding.decode (huffman.py:121-139): prefix walk; trailing bits that end no code are dropped,
// characters other than '0' / '1' extend the current code without matching (as in the reference)
extern "C" int tmae_huffman_decode(const char* bits, long long nbits, const int64_t* syms, const int32_t* lens,
                                   const uint64_t* codes, int nsym, int64_t* out, long long cap, long long* nout) {
  if ((!bits && nbits > 0) || !syms || !lens || !codes || !nout || nsym <= 0) {
    tmae_set_error(TMAE_EINVAL, "tmae_huffman_decode: bad arguments");
    return TMAE_EINVAL;
  }
  // decoding trie over the code table
  std::vector<int> child0(1, -1), child1(1, -1), leaf(1, -1);
  for (int i = 0; i < nsym; ++i) {
    int node = 0;
    for (int b = lens[i] - 1; b >= 0; --b) {
      std::vector<int>& ch = ((codes[i] >> b) & 1u) ? child1 : child0;
      if (ch[node] < 0) {
        ch[node] = (int)leaf.size();
        child0.push_back(-1);
        child1.push_back(-1);
        leaf.push_back(-1);
      }
      node = ch[node];
    }
    leaf[node] = i;
  }
  long long n = 0;
  int node = 0;
  bool dead = false;  // a non-binary character: the reference's current_code can never match again
  for (long long p = 0; p < nbits && !dead; ++p) {
    const char c = bits[p];
    if (c != '0' && c != '1') {
      dead = true;
      break;
    }
    node = (c == '1') ? child1[node] : child0[node];
    if (node < 0) {
      dead = true;
      break;
    }
    if (leaf[node] >= 0) {
      if (n >= cap) {
        tmae_set_error(TMAE_EINVAL, "tmae_huffman_decode: output buffer too small");
        return TMAE_EINVAL;
      }
      out[n++] = syms[leaf[node]];
      node = 0;
    }
  }
  *nout = n;
  return TMAE_OK;
}
