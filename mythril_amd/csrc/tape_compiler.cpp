// tape_compiler.cpp — boundary tape (mq.h DAG) -> register-stack program for the gfx950 kernels.
//
// Pipeline (per tape):
//   1. validate + sort-check the DAG (postfix, operands precede users);
//   2. rewrite to an internal DAG: select over store chains / K(v) becomes an ite chain
//      (select(store(A,k,v),i) = i==k ? v : select(A,i)), select over an
//      array variable becomes a table lookup (G_UF1), predicates get reversed twins so the
//      scheduler may evaluate either operand first;
//   3. hoist every non-leaf node with >1 user into an LDS temp (liveness-based slot reuse);
//   4. emit stack code with Sethi-Ullman operand ordering for commutative ops, so the
//      register stack stays shallow (handlers are specialized per stack slot).
#include "tape_compiler.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <tuple>
#include <unordered_map>

namespace mq {

static inline int nl_of(int w) { return w == 0 ? 1 : (w + 31) / 32; }

namespace {

enum Kind { K_BOOL, K_BV, K_ARRAY };

struct INode {
  uint32_t gop = 0;
  int width = 0;       // result width (0 = Bool)
  uint32_t imm = 0;    // primary immediate
  uint32_t imm2 = 0;   // secondary immediate (second word)
  int kid[3] = {-1, -1, -1};
  int nk = 0;
  bool leaf = false;
  bool commut = false;
  uint32_t rev_gop = 0;  // op to use when operands are swapped (0 = not swappable)
};

struct Key {
  uint32_t gop, imm, imm2;
  int w, k0, k1, k2;
  bool operator==(const Key& o) const {
    return gop == o.gop && imm == o.imm && imm2 == o.imm2 && w == o.w && k0 == o.k0 && k1 == o.k1 && k2 == o.k2;
  }
};

struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint64_t v : {(uint64_t)k.gop, (uint64_t)k.imm, (uint64_t)k.imm2, (uint64_t)(uint32_t)k.w, (uint64_t)(uint32_t)k.k0,
                       (uint64_t)(uint32_t)k.k1, (uint64_t)(uint32_t)k.k2})
      h = (h ^ v) * 0x100000001B3ull + (h >> 29);
    return (size_t)h;
  }
};

// hash-consing of the internal DAG: an open-addressing table of node indices keyed by
// (op, immediates, width, kids) — one probe per node, no allocation per entry (the ordered map
// it replaces was 40 % of a drop-in batch's compile time)
struct Builder {
  std::vector<INode> nodes;
  std::vector<int> table;   // node index + 1, 0 = empty; size a power of two
  static Key key_of(const INode& n) { return Key{n.gop, n.imm, n.imm2, n.width, n.kid[0], n.kid[1], n.kid[2]}; }
  void reserve(size_t n) {
    nodes.reserve(n);
    size_t sz = 64;
    while (sz < 2 * n) sz <<= 1;
    table.assign(sz, 0);
  }
  void grow() {
    std::vector<int> old(table.size() * 2, 0);
    old.swap(table);
    const size_t mask = table.size() - 1;
    for (int v : old)
      if (v) {
        size_t h = KeyHash()(key_of(nodes[v - 1])) & mask;
        while (table[h]) h = (h + 1) & mask;
        table[h] = v;
      }
  }
  int add(const INode& n) {
    if (table.empty()) reserve(64);
    const Key k = key_of(n);
    const size_t mask = table.size() - 1;
    size_t h = KeyHash()(k) & mask;
    while (int v = table[h]) {
      if (key_of(nodes[v - 1]) == k) return v - 1;
      h = (h + 1) & mask;
    }
    nodes.push_back(n);
    table[h] = (int)nodes.size();
    if (2 * nodes.size() > table.size()) grow();
    return (int)nodes.size() - 1;
  }
};

INode mk(uint32_t gop, int w, std::initializer_list<int> kids, uint32_t imm = 0, uint32_t imm2 = 0) {
  INode n;
  n.gop = gop;
  n.width = w;
  n.imm = imm;
  n.imm2 = imm2;
  for (int k : kids) n.kid[n.nk++] = k;
  return n;
}

struct WordsHash {
  size_t operator()(const std::vector<uint32_t>& w) const {
    uint64_t h = 0xCBF29CE484222325ull;
    for (uint32_t x : w) h = (h ^ x) * 0x100000001B3ull;
    return (size_t)h;
  }
};

struct Fail {
  std::string why;
};

}  // namespace

CompiledTape compile_tape(const mq_tape_batch* batch, int32_t t, const CompileLimits& lim) {
  CompiledTape out;
  const int64_t base = batch->tape_offsets[t];
  const int64_t nn = batch->tape_offsets[t + 1] - base;
  out.n_nodes = (uint32_t)nn;
  if (nn <= 0) {
    out.why = "empty tape";
    return out;
  }
  const mq_node* nd = batch->nodes + base;
  try {
    // ---------------------------------------------------------------- 1. validate, kinds, widths
    std::vector<Kind> kind(nn);
    std::vector<uint32_t> chunk_k(nn, 0);   // MQ_OP_UF_CHUNK: the key chunk's index
    int maxw = 1;
    auto ref = [&](int64_t i, uint32_t r) -> int {
      if (r >= (uint32_t)i) throw Fail{"operand does not precede its user"};
      return (int)r;
    };
    for (int64_t i = 0; i < nn; i++) {
      const mq_node& n = nd[i];
      if (n.width > maxw) maxw = n.width;
      switch (n.op) {
        case MQ_OP_STORE:
        case MQ_OP_CONST_ARRAY:
        case MQ_OP_ARRAY_VAR:
          kind[i] = K_ARRAY;
          break;
        case MQ_OP_SELECT:
        case MQ_OP_UF:
        case MQ_OP_UF_WIDE:
        case MQ_OP_VAR:
          kind[i] = n.width == 0 ? K_BOOL : K_BV;
          break;
        case MQ_OP_TRUE: case MQ_OP_FALSE: case MQ_OP_NOT: case MQ_OP_AND: case MQ_OP_OR:
        case MQ_OP_XOR: case MQ_OP_IMPLIES: case MQ_OP_IFF: case MQ_OP_BITE: case MQ_OP_EQ:
        case MQ_OP_ULT: case MQ_OP_ULE: case MQ_OP_SLT: case MQ_OP_SLE: case MQ_OP_UMUL_NOOVFL:
        case MQ_OP_SMUL_NOOVFL: case MQ_OP_SMUL_NOUDFL:
          kind[i] = K_BOOL;
          break;
        default:
          kind[i] = K_BV;
      }
      // operand references (sort checks are light: the host builder enforces full sorts)
      switch (n.op) {
        case MQ_OP_CONST:
          if ((int64_t)n.a + nl_of(n.width) > batch->n_const_words) throw Fail{"const out of pool"};
          break;
        case MQ_OP_VAR: case MQ_OP_TRUE: case MQ_OP_FALSE: case MQ_OP_ARRAY_VAR:
          break;
        case MQ_OP_NOT: case MQ_OP_NEG: case MQ_OP_BNOT: case MQ_OP_EXTRACT: case MQ_OP_ZEXT:
        case MQ_OP_SEXT: case MQ_OP_CONST_ARRAY: case MQ_OP_KECCAK:
          ref(i, n.a);
          break;
        case MQ_OP_BITE: case MQ_OP_ITE: case MQ_OP_STORE:
          ref(i, n.a); ref(i, n.b); ref(i, n.c);
          break;
        case MQ_OP_UF:
          ref(i, n.b);
          if (n.c != MQ_NONE) ref(i, n.c);
          break;
        case MQ_OP_UF_CHUNK:
          ref(i, n.b);
          if (n.width != 64 || nd[n.b].width == 0 || nd[n.b].width > 256) throw Fail{"bad UF key chunk"};
          if (n.c != MQ_NONE) {
            ref(i, n.c);
            if (nd[n.c].op != MQ_OP_UF_CHUNK || nd[n.c].a != n.a) throw Fail{"bad UF key chunk chain"};
            chunk_k[i] = chunk_k[n.c] + 1;
          }
          break;
        case MQ_OP_UF_WIDE:
          ref(i, n.b);
          if (nd[n.b].op != MQ_OP_UF_CHUNK || nd[n.b].a != n.a) throw Fail{"UF_WIDE without its key chunks"};
          if (std::find(out.wide_funcs.begin(), out.wide_funcs.end(), n.a) == out.wide_funcs.end())
            out.wide_funcs.push_back(n.a);
          break;
        default:
          if (n.op > 100) throw Fail{"unknown opcode"};
          ref(i, n.a); ref(i, n.b);
      }
      if (n.op == MQ_OP_EQ && kind[n.a] == K_ARRAY) throw Fail{"array equality"};
      if ((n.op == MQ_OP_EQ || n.op == MQ_OP_ULT || n.op == MQ_OP_ULE || n.op == MQ_OP_SLT || n.op == MQ_OP_SLE ||
           n.op == MQ_OP_UMUL_NOOVFL || n.op == MQ_OP_SMUL_NOOVFL || n.op == MQ_OP_SMUL_NOUDFL) &&
          nd[n.a].width != nd[n.b].width)
        throw Fail{"predicate operand width mismatch"};
      if (n.op == MQ_OP_KECCAK) {
        const int aw = nd[n.a].width;
        if (aw == 0 || aw % 8 || aw > kMaxWidth || n.width != 256) throw Fail{"keccak argument must be 8..2048 bits, bytes"};
        out.keccak = true;
      }
      // multiplication, division and the multiplication-overflow predicates run on at most 16
      // limbs (qs_kernels.hip kArithLimbs); Mythril only builds them at 256 / 257 bits
      if ((n.op == MQ_OP_MUL || n.op == MQ_OP_UDIV || n.op == MQ_OP_UREM || n.op == MQ_OP_SDIV ||
           n.op == MQ_OP_SREM || n.op == MQ_OP_SMOD) && n.width > 512)
        throw Fail{"multiplication / division wider than 512 bits"};
      if ((n.op == MQ_OP_UMUL_NOOVFL || n.op == MQ_OP_SMUL_NOOVFL || n.op == MQ_OP_SMUL_NOUDFL) && nd[n.a].width > 512)
        throw Fail{"overflow predicate wider than 512 bits"};
    }
    if (kind[nn - 1] != K_BOOL && !(lim.value_root && kind[nn - 1] == K_BV)) throw Fail{"root is not Bool"};
    // limbs per stack slot: the widest value of the tape (interpreted keccak runs on L >= 16)
    if (maxw <= 256 && !out.keccak) out.L = 8;
    else if (maxw <= 512) out.L = 16;
    else if (maxw <= 1024) out.L = 32;
    else if (maxw <= kMaxWidth) out.L = 64;
    else throw Fail{"width > 2048"};
    const int L = out.L;
    const int max_depth = L == 8 ? lim.max_depth_l8 : L == 16 ? lim.max_depth_l16 : L == 32 ? lim.max_depth_l32 : lim.max_depth_l64;
    const int max_temps = L == 8 ? lim.max_temps_l8 : L == 16 ? lim.max_temps_l16 : L == 32 ? lim.max_temps_l32 : lim.max_temps_l64;

    // ---------------------------------------------------------------- 2. internal DAG
    Builder B;
    B.reserve((size_t)nn * 2);
    std::vector<int> map(nn, -1);
    std::unordered_map<std::vector<uint32_t>, uint32_t, WordsHash> cmemo;  // constant dedup -> word offset
    auto konst = [&](int64_t i) -> int {
      const mq_node& n = nd[i];
      std::vector<uint32_t> w(L, 0);
      for (int k = 0; k < nl_of(n.width); k++) w[k] = batch->const_words[n.a + k];
      if (n.width % 32) w[nl_of(n.width) - 1] &= (1u << (n.width % 32)) - 1u;
      uint32_t off;
      auto it = cmemo.find(w);
      if (it == cmemo.end()) {
        off = (uint32_t)out.consts.size();
        out.consts.insert(out.consts.end(), w.begin(), w.end());
        cmemo[w] = off;
      } else {
        off = it->second;
      }
      if (off > (uint32_t)kMaxImm) throw Fail{"too many constants"};
      INode x = mk(G_PUSH_CONST, n.width, {}, off);
      x.leaf = true;
      return B.add(x);
    };
    // select(array node arr, index internal node idx)
    std::function<int(int64_t, int, int)> select = [&](int64_t arr, int idx, int rw) -> int {
      const mq_node& a = nd[arr];
      if (a.op == MQ_OP_STORE) {
        int key = map[a.b], val = map[a.c];
        int cond = B.add([&] { INode e = mk(G_EQ, 0, {idx, key}, (uint32_t)nd[a.b].width); e.commut = true; return e; }());
        int rest = select(a.a, idx, rw);
        return B.add(mk(rw == 0 ? G_BITE : G_ITE, rw, {cond, val, rest}, (uint32_t)rw));
      }
      if (a.op == MQ_OP_CONST_ARRAY) return map[a.a];
      if (a.op == MQ_OP_ARRAY_VAR) return B.add(mk(G_UF1, rw, {idx}, a.a, (uint32_t)rw));
      if (a.op == MQ_OP_ITE || a.op == MQ_OP_BITE) throw Fail{"ite over arrays"};
      throw Fail{"unsupported array term"};
    };
    for (int64_t i = 0; i < nn; i++) {
      const mq_node& n = nd[i];
      int w = n.width;
      auto A = [&]() { return map[n.a]; };
      auto Bk = [&]() { return map[n.b]; };
      auto Ck = [&]() { return map[n.c]; };
      auto bin = [&](uint32_t g, bool commut, uint32_t rev, uint32_t imm) {
        INode x = mk(g, w, {A(), Bk()}, imm);
        x.commut = commut;
        x.rev_gop = rev;
        return B.add(x);
      };
      int aw = (n.op != MQ_OP_VAR && n.op != MQ_OP_CONST && n.op != MQ_OP_TRUE && n.op != MQ_OP_FALSE &&
                n.op != MQ_OP_ARRAY_VAR && n.op != MQ_OP_UF && n.op != MQ_OP_UF_CHUNK && n.op != MQ_OP_UF_WIDE &&
                n.a < (uint32_t)i)
                   ? nd[n.a].width : 0;
      int r = -1;
      switch (n.op) {
        case MQ_OP_CONST: r = konst(i); break;
        case MQ_OP_VAR: {
          if (n.a > (uint32_t)kMaxImm) throw Fail{"var index too large"};
          INode x = mk(w == 0 ? G_PUSH_VAR_B : G_PUSH_VAR, w, {}, n.a);
          x.leaf = true;
          r = B.add(x);
          break;
        }
        case MQ_OP_TRUE: case MQ_OP_FALSE: {
          INode x = mk(G_PUSH_BOOL, 0, {}, n.op == MQ_OP_TRUE ? 1u : 0u);
          x.leaf = true;
          r = B.add(x);
          break;
        }
        case MQ_OP_NOT: r = B.add(mk(G_NOT, 0, {A()})); break;
        case MQ_OP_AND: r = bin(G_AND, true, G_AND, 0); break;
        case MQ_OP_OR: r = bin(G_OR, true, G_OR, 0); break;
        case MQ_OP_XOR: r = bin(G_XOR, true, G_XOR, 0); break;
        case MQ_OP_IFF: r = bin(G_IFF, true, G_IFF, 0); break;
        case MQ_OP_IMPLIES: r = bin(G_IMPLIES, false, 0, 0); break;
        case MQ_OP_BITE: r = B.add(mk(G_BITE, 0, {A(), Bk(), Ck()})); break;
        case MQ_OP_EQ: r = bin(G_EQ, true, G_EQ, aw); break;
        case MQ_OP_ULT: r = bin(G_ULT, true, G_UGT, aw); break;
        case MQ_OP_ULE: r = bin(G_ULE, true, G_UGE, aw); break;
        case MQ_OP_SLT: r = bin(G_SLT, true, G_SGT, aw); break;
        case MQ_OP_SLE: r = bin(G_SLE, true, G_SGE, aw); break;
        case MQ_OP_UMUL_NOOVFL: r = bin(G_UMUL_NOOVFL, true, G_UMUL_NOOVFL, aw); break;
        case MQ_OP_SMUL_NOOVFL: r = bin(G_SMUL_NOOVFL, true, G_SMUL_NOOVFL, aw); break;
        case MQ_OP_SMUL_NOUDFL: r = bin(G_SMUL_NOUDFL, true, G_SMUL_NOUDFL, aw); break;
        case MQ_OP_ADD: r = bin(G_ADD, true, G_ADD, w); break;
        case MQ_OP_SUB: r = bin(G_SUB, false, 0, w); break;
        case MQ_OP_MUL: r = bin(G_MUL, true, G_MUL, w); break;
        case MQ_OP_NEG: r = B.add(mk(G_NEG, w, {A()}, w)); break;
        case MQ_OP_UDIV: r = bin(G_UDIV, false, 0, w); break;
        case MQ_OP_UREM: r = bin(G_UREM, false, 0, w); break;
        case MQ_OP_SDIV: r = bin(G_SDIV, false, 0, w); break;
        case MQ_OP_SREM: r = bin(G_SREM, false, 0, w); break;
        case MQ_OP_SMOD: r = bin(G_SMOD, false, 0, w); break;
        case MQ_OP_BAND: r = bin(G_BAND, true, G_BAND, w); break;
        case MQ_OP_BOR: r = bin(G_BOR, true, G_BOR, w); break;
        case MQ_OP_BXOR: r = bin(G_BXOR, true, G_BXOR, w); break;
        case MQ_OP_BNOT: r = B.add(mk(G_BNOT, w, {A()}, w)); break;
        case MQ_OP_SHL: r = bin(G_SHL, false, 0, w); break;
        case MQ_OP_LSHR: r = bin(G_LSHR, false, 0, w); break;
        case MQ_OP_ASHR: r = bin(G_ASHR, false, 0, w); break;
        case MQ_OP_EXTRACT: {
          if ((int)n.b - (int)n.c + 1 != w || n.b >= (uint32_t)aw) throw Fail{"bad extract"};
          r = (n.c == 0 && w == aw) ? A() : B.add(mk(G_EXTRACT, w, {A()}, n.c, (uint32_t)w));
          break;
        }
        case MQ_OP_CONCAT: {
          int bw = nd[n.b].width;
          if (aw + bw != w) throw Fail{"bad concat"};
          r = B.add(mk(G_CONCAT, w, {A(), Bk()}, (uint32_t)bw, (uint32_t)w));
          break;
        }
        case MQ_OP_ZEXT: r = A(); break;  // canonical values are already zero-extended
        case MQ_OP_SEXT: r = B.add(mk(G_SEXT, w, {A()}, (uint32_t)aw, (uint32_t)w)); break;
        case MQ_OP_ITE: r = B.add(mk(G_ITE, w, {A(), Bk(), Ck()}, w)); break;
        case MQ_OP_STORE: case MQ_OP_CONST_ARRAY: case MQ_OP_ARRAY_VAR: r = -1; break;
        case MQ_OP_KECCAK: r = B.add(mk(G_KECCAK, 256, {A()}, (uint32_t)aw)); break;
        case MQ_OP_SELECT: r = select(n.a, Bk(), w); break;
        case MQ_OP_UF: {
          if (n.a > (uint32_t)kMaxImm) throw Fail{"function id too large"};
          if (n.c == MQ_NONE) r = B.add(mk(G_UF1, w, {Bk()}, n.a, (uint32_t)w));
          else r = B.add(mk(G_UF2, w, {Bk(), Ck()}, n.a, (uint32_t)w));
          break;
        }
        case MQ_OP_UF_CHUNK: {
          if (n.a > (uint32_t)kMaxImm) throw Fail{"function id too large"};
          if (n.c == MQ_NONE) r = B.add(mk(G_UFK0, 64, {Bk()}, n.a, 0u));
          else r = B.add(mk(G_UFK, 64, {Ck(), Bk()}, n.a, chunk_k[i]));
          break;
        }
        case MQ_OP_UF_WIDE: {
          if (n.a > (uint32_t)kMaxImm) throw Fail{"function id too large"};
          r = B.add(mk(G_UFKV, w, {Bk()}, n.a, (uint32_t)w));
          break;
        }
        default:
          throw Fail{"unsupported opcode"};
      }
      map[i] = r;
    }
    const int root = map[nn - 1];
    if (root < 0) throw Fail{"root lowered to nothing"};

    // ---------------------------------------------------------------- 3. reachability, uses, hoisting
    const int NI = (int)B.nodes.size();
    std::vector<int> uses(NI, 0);
    std::vector<char> live(NI, 0);
    {
      std::vector<int> st{root};
      live[root] = 1;
      while (!st.empty()) {
        int x = st.back();
        st.pop_back();
        for (int k = 0; k < B.nodes[x].nk; k++) {
          int c = B.nodes[x].kid[k];
          uses[c]++;
          if (!live[c]) {
            live[c] = 1;
            st.push_back(c);
          }
        }
      }
    }
    // Phases 3-4 as one function of the spill limit: spill > 0 additionally hoists subtrees into
    // temps until every unit needs at most `spill` stack slots (Sethi-Ullman order; the G
    // assembly interpreter has kQsaStackG slots, the P / C++ kernels more).
    auto build = [&](int spill, std::vector<uint32_t>& prog, int& depth_out, int& temps_out) {
    std::vector<char> hoist(NI, 0);
    // Rematerialisation: a shared node whose expression is tiny and cheap (a calldata byte
    // `ite(slt(i, size), cd_i, 0)`, a masked extract) is re-evaluated at each use instead of
    // occupying a temp slot: temps cost 2 KB per wave and their count bounds what compiles.
    // remat_cost(x) = nodes re-emitted per extra use (hoisted kids and leaves are free pushes).
    std::vector<int> remat_cost(NI, 0);
    auto expensive = [&](uint32_t g) {
      return g == G_MUL || g == G_UDIV || g == G_UREM || g == G_SDIV || g == G_SREM || g == G_SMOD ||
             g == G_UF1 || g == G_UF2 || g == G_UFK0 || g == G_UFK || g == G_UFKV || g == G_KECCAK ||
             g == G_UMUL_NOOVFL || g == G_SMUL_NOOVFL ||
             g == G_SMUL_NOUDFL || g == G_SHL || g == G_LSHR || g == G_ASHR;
    };
    for (int x = 0; x < NI; x++) {
      if (!live[x]) continue;
      const INode& n = B.nodes[x];
      if (n.leaf) continue;
      int c = expensive(n.gop) ? 1000 : 1;
      for (int k = 0; k < n.nk; k++) {
        const int kid = n.kid[k];
        if (!B.nodes[kid].leaf && !hoist[kid]) c += remat_cost[kid];
      }
      remat_cost[x] = c;
      if (x != root && uses[x] > 1 && c > lim.remat_max_nodes) hoist[x] = 1;
    }

    // stack need with hoisted nodes as leaves (Sethi-Ullman)
    std::vector<int> need(NI, 1);
    std::vector<char> swap(NI, 0);
    // need[x] depends on its kids only (lower indices): recompute from the lowest changed node
    auto compute_need = [&](int from) {
    for (int x = from; x < NI; x++) {
      if (!live[x]) continue;
      const INode& n = B.nodes[x];
      swap[x] = 0;
      auto nd_of = [&](int c) { return (hoist[c] || B.nodes[c].leaf) ? 1 : need[c]; };
      if (n.leaf || n.nk == 0) need[x] = 1;
      else if (n.nk == 1) need[x] = nd_of(n.kid[0]);
      else if (n.nk == 2) {
        int a = nd_of(n.kid[0]), b = nd_of(n.kid[1]);
        int fwd = std::max(a, b + 1), bwd = std::max(b, a + 1);
        // tie: put a variable leaf second, where the assembly interpreter fuses its push into
        // the operation (gen_qsa.py ...V handlers)
        auto is_var = [&](int c) { return !hoist[c] && B.nodes[c].leaf && B.nodes[c].gop == G_PUSH_VAR; };
        const bool var_second = bwd == fwd && is_var(n.kid[0]) && !is_var(n.kid[1]);
        if (n.rev_gop && (bwd < fwd || var_second)) {
          swap[x] = 1;
          need[x] = bwd;
        } else {
          need[x] = fwd;
        }
      } else {
        const int c0 = nd_of(n.kid[0]), c1 = nd_of(n.kid[1]), c2 = nd_of(n.kid[2]);
        const int fwd = std::max({c0, c1 + 1, c2 + 2});
        const int ef = std::max({c2, c0 + 1, c1 + 2});  // else, cond, then
        if ((n.gop == G_ITE || n.gop == G_BITE) && ef < fwd) {
          swap[x] = 1;
          need[x] = ef;
        } else {
          need[x] = fwd;
        }
      }
    }
    };
    compute_need(0);
    if (spill > 0) {
      // the lowest (first in topological order) unit node needing more than `spill` slots has
      // kids that each fit: hoist its deepest kid into a temp, recompute, repeat.  (With
      // spill >= 3 such a node always has a non-leaf kid: all-leaf operands need <= 3 slots.)
      // (nodes below the last bad one fit and stay so: hoisting only lowers needs)
      int scan = 0;
      for (;;) {
        int bad = -1;
        for (int x = scan; x < NI && bad < 0; x++)
          if (live[x] && !B.nodes[x].leaf && need[x] > spill) bad = x;
        if (bad < 0) break;
        const INode& n = B.nodes[bad];
        int best = -1;
        for (int k = 0; k < n.nk; k++) {
          const int c = n.kid[k];
          if (hoist[c] || B.nodes[c].leaf) continue;
          if (best < 0 || need[c] > need[best]) best = c;
        }
        if (best < 0) throw Fail{"cannot spill"};
        hoist[best] = 1;
        compute_need(best);
        scan = bad;
      }
    }
    std::vector<int> units;  // hoisted nodes in topological (index) order, then root
    for (int x = 0; x < NI; x++)
      if (live[x] && hoist[x] && x != root) units.push_back(x);
    units.push_back(root);

    // temp slot allocation with reuse after last use
    std::vector<int> unit_of_last_use(NI, -1);
    std::vector<std::vector<int>> refs(units.size());
    std::vector<int> vis(NI, -1);   // unit that last visited the node
    for (size_t u = 0; u < units.size(); u++) {
      // temps referenced by unit u: hoisted nodes reachable from units[u] without crossing hoisted nodes
      std::vector<int> st;
      int top = units[u];
      for (int k = 0; k < B.nodes[top].nk; k++) st.push_back(B.nodes[top].kid[k]);
      while (!st.empty()) {
        int x = st.back();
        st.pop_back();
        if (vis[x] == (int)u) continue;
        vis[x] = (int)u;
        if (hoist[x]) {
          refs[u].push_back(x);
          unit_of_last_use[x] = (int)u;
          continue;
        }
        for (int k = 0; k < B.nodes[x].nk; k++) st.push_back(B.nodes[x].kid[k]);
      }
    }
    std::vector<int> slot(NI, -1);
    std::vector<int> free_slots;
    int n_slots = 0;

    // ---------------------------------------------------------------- 4. emission
    int maxd = 0;
    auto emit_rec = [&](auto& emit_self, int x, int d) -> void {
      auto emit = [&](int x2, int d2) { emit_self(emit_self, x2, d2); };
      if (d >= max_depth) throw Fail{"stack too deep"};
      maxd = std::max(maxd, d + 1);
      const INode& n = B.nodes[x];
      if (hoist[x] && slot[x] >= 0) {
        prog.push_back(gword(n.width == 0 ? G_PUSH_TMP_B : G_PUSH_TMP, d, slot[x]));
        return;
      }
      if (n.leaf) {
        prog.push_back(gword(n.gop, d, n.imm));
        return;
      }
      uint32_t g = n.gop;
      if (n.nk == 1) {
        emit(n.kid[0], d);
      } else if (n.nk == 2) {
        if (swap[x]) {
          emit(n.kid[1], d);
          emit(n.kid[0], d + 1);
          g = n.rev_gop;
        } else {
          emit(n.kid[0], d);
          emit(n.kid[1], d + 1);
        }
        d += 1;
      } else if (n.nk == 3) {
        if (swap[x]) {
          emit(n.kid[2], d);
          emit(n.kid[0], d + 1);
          emit(n.kid[1], d + 2);
          g = n.gop == G_ITE ? G_ITE_EF : G_BITE_EF;
        } else {
          emit(n.kid[0], d);
          emit(n.kid[1], d + 1);
          emit(n.kid[2], d + 2);
        }
        d += 2;
      }
      if (n.imm > (uint32_t)kMaxImm) throw Fail{"immediate too large"};
      prog.push_back(gword(g, d, n.imm));
      if (has_imm2(g)) prog.push_back(n.imm2);
    };
    for (size_t u = 0; u < units.size(); u++) {
      int x = units[u];
      emit_rec(emit_rec, x, 0);
      // release temps whose last use was this unit (before allocating this unit's own slot)
      for (int r : refs[u])
        if (unit_of_last_use[r] == (int)u) free_slots.push_back(slot[r]);
      if (x != root) {
        int s;
        if (!free_slots.empty()) {
          s = free_slots.back();
          free_slots.pop_back();
        } else {
          s = n_slots++;
        }
        slot[x] = s;
        prog.push_back(gword(B.nodes[x].width == 0 ? G_STORE_TMP_B : G_STORE_TMP, 0, s));
      }
    }
    if (n_slots > max_temps) throw Fail{"too many temps"};
    prog.push_back(gword(G_END, 0, 0));
    depth_out = maxd;
    temps_out = n_slots;
    };
    build(0, out.prog, out.depth, out.n_temps);
    // the G assembly interpreter's stack is shallower: a spilled variant for it (a failure only
    // leaves the tape to the other kernels)
    if (lim.g_depth > 0 && out.depth > lim.g_depth) {
      try {
        build(lim.g_depth, out.prog_g, out.depth_g, out.n_temps_g);
      } catch (const Fail&) {
        out.prog_g.clear();
        out.depth_g = 0;
        out.n_temps_g = 0;
      }
    }
    out.supported = true;
  } catch (const Fail& f) {
    out.supported = false;
    out.why = f.why;
    out.prog.clear();
    out.prog_g.clear();
    out.wide_funcs.clear();
    out.consts.clear();
  }
  out.alg_ops = tape_alg_ops(batch, t);
  return out;
}

double tape_alg_ops(const mq_tape_batch* batch, int32_t t) {
  const int64_t base = batch->tape_offsets[t];
  const int64_t nn = batch->tape_offsets[t + 1] - base;
  const mq_node* nd = batch->nodes + base;
  double ops = 0;
  for (int64_t i = 0; i < nn; i++) {
    const mq_node& n = nd[i];
    double L = nl_of(n.width);
    double La = (n.a < (uint32_t)i) ? nl_of(nd[n.a].width) : L;
    switch (n.op) {
      case MQ_OP_CONST: case MQ_OP_VAR: case MQ_OP_TRUE: case MQ_OP_FALSE:
      case MQ_OP_STORE: case MQ_OP_CONST_ARRAY: case MQ_OP_ARRAY_VAR: case MQ_OP_ZEXT:
        break;
      case MQ_OP_NOT: case MQ_OP_AND: case MQ_OP_OR: case MQ_OP_XOR: case MQ_OP_IMPLIES:
      case MQ_OP_IFF: case MQ_OP_BITE:
        ops += 1;
        break;
      case MQ_OP_EQ: case MQ_OP_ULT: case MQ_OP_ULE: case MQ_OP_SLT: case MQ_OP_SLE:
        ops += La;
        break;
      case MQ_OP_UMUL_NOOVFL: case MQ_OP_SMUL_NOOVFL: case MQ_OP_SMUL_NOUDFL:
        ops += 2 * La * La;
        break;
      case MQ_OP_ADD: case MQ_OP_SUB: case MQ_OP_NEG: case MQ_OP_BAND: case MQ_OP_BOR:
      case MQ_OP_BXOR: case MQ_OP_BNOT: case MQ_OP_ITE:
        ops += L;
        break;
      case MQ_OP_EXTRACT: case MQ_OP_CONCAT: case MQ_OP_SEXT:
        ops += L;
        break;
      case MQ_OP_SHL: case MQ_OP_LSHR: case MQ_OP_ASHR:
        ops += 2 * L;
        break;
      case MQ_OP_MUL:
        ops += L * (L + 1);
        break;
      case MQ_OP_UDIV: case MQ_OP_UREM:
        ops += 2 * L * L + 8 * L;
        break;
      case MQ_OP_SDIV: case MQ_OP_SREM: case MQ_OP_SMOD:
        ops += 2 * L * L + 12 * L;
        break;
      case MQ_OP_SELECT: {
        // c * (L_key + L_val) over the store chain, + one table lookup at its base
        uint32_t arr = n.a;
        double Lk = nl_of(nd[n.b].width);
        while (arr < (uint32_t)i && nd[arr].op == MQ_OP_STORE) {
          ops += Lk + L;
          arr = nd[arr].a;
        }
        if (arr < (uint32_t)i && nd[arr].op == MQ_OP_ARRAY_VAR) ops += Lk + L;
        break;
      }
      case MQ_OP_UF: {
        double Larg = (n.b < (uint32_t)i ? nl_of(nd[n.b].width) : 8) + (n.c != MQ_NONE && n.c < (uint32_t)i ? nl_of(nd[n.c].width) : 0);
        ops += Larg + L;  // one-entry table (model-dependent; SURVEY §8(d) e*L_arg + L_val, e = 1)
        break;
      }
      case MQ_OP_UF_CHUNK:   // the key's share of the lookup, chunk by chunk (e = 1, as MQ_OP_UF)
        ops += n.b < (uint32_t)i ? nl_of(nd[n.b].width) : 8;
        break;
      case MQ_OP_UF_WIDE:
        ops += L;
        break;
      case MQ_OP_KECCAK:
        // keccak-f[1600] permutations: one per started 136-byte block (the pad byte included)
        ops += kKeccakOpsPerBlock * std::floor(((n.a < (uint32_t)i ? nd[n.a].width / 8.0 : La * 4) + 1 + 135) / 136);
        break;
      default:
        return -1;
    }
  }
  return ops;
}

}  // namespace mq
