// Minimal GoogleTest-compatible shim (TEST, TEST_P, INSTANTIATE_TEST_SUITE_P, EXPECT_*), enough to build the
// reference's sw/tests/*.cpp unmodified against libgcow.so. Test infrastructure; written for this repository.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <sstream>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace testing {
namespace internal {
inline int& failures() { static int f = 0; return f; }
inline bool& current_failed() { static bool f = false; return f; }
struct Case { std::string name; std::function<void()> fn; };
inline std::vector<Case>& registry() { static std::vector<Case> r; return r; }
struct Registrar {
  Registrar(const char* suite, const char* name, std::function<void()> fn)
  {
    registry().push_back({std::string(suite) + "." + name, fn});
  }
};
struct Msg {
  bool active;
  std::ostringstream os;
  explicit Msg(bool a) : active(a) {}
  template <class T> Msg& operator<<(const T& v) { if (active) os << v; return *this; }
  ~Msg() { if (active && !os.str().empty()) std::cout << "  note: " << os.str() << std::endl; }
};
template <class A, class B>
bool eq(const A& a, const B& b, const char* ea, const char* eb, const char* file, int line)
{
  if (a == b) return true;
  std::cout << file << ":" << line << ": Failure: expected " << ea << " == " << eb << "  (" << a << " vs " << b
            << ")" << std::endl;
  current_failed() = true;
  return false;
}
inline bool truth(bool v, bool want, const char* e, const char* file, int line)
{
  if (v == want) return true;
  std::cout << file << ":" << line << ": Failure: " << e << " is " << (v ? "true" : "false") << std::endl;
  current_failed() = true;
  return false;
}
// TEST_P plumbing: bodies registered per fixture, run for every instantiated value.
template <class F> struct ParamBodies {
  static std::vector<std::pair<std::string, std::function<void()>>>& get()
  {
    static std::vector<std::pair<std::string, std::function<void()>>> v;
    return v;
  }
};
}  // namespace internal

class Test {
 public:
  virtual ~Test() {}
  virtual void TestBody() = 0;
};

template <class T> class TestWithParam : public Test {
 public:
  typedef T ParamType;
  static const T*& param() { static const T* p = nullptr; return p; }
  const T& GetParam() const { return *param(); }
};

template <class... V> std::vector<std::tuple<int>> Values(V... v) { return {std::tuple<int>(v)...}; }

inline void InitGoogleTest(int*, char**) {}
}  // namespace testing

inline int RUN_ALL_TESTS()
{
  using namespace testing::internal;
  int n = 0;
  for (auto& c : registry()) {
    current_failed() = false;
    std::cout << "[ RUN      ] " << c.name << std::endl;
    c.fn();
    std::cout << (current_failed() ? "[  FAILED  ] " : "[       OK ] ") << c.name << std::endl;
    failures() += current_failed() ? 1 : 0;
    n++;
  }
  std::cout << "[==========] " << n << " tests ran, " << failures() << " failed." << std::endl;
  return failures() ? 1 : 0;
}

#define GCOW_SHIM_CAT_(a, b) a##b
#define GCOW_SHIM_CAT(a, b) GCOW_SHIM_CAT_(a, b)

#define TEST(suite, name)                                                                          \
  static void GCOW_SHIM_CAT(suite##_##name, _body)();                                             \
  static ::testing::internal::Registrar GCOW_SHIM_CAT(suite##_##name, _reg)(#suite, #name,        \
                                                                            &GCOW_SHIM_CAT(suite##_##name, _body)); \
  static void GCOW_SHIM_CAT(suite##_##name, _body)()

#define TEST_P(fixture, name)                                                                      \
  struct fixture##_##name##_Test : public fixture {                                                \
    void TestBody() override;                                                                      \
  };                                                                                               \
  static int fixture##_##name##_reg = (::testing::internal::ParamBodies<fixture>::get().push_back( \
                                           {#name, [] { fixture##_##name##_Test t; t.TestBody(); }}), 0); \
  void fixture##_##name##_Test::TestBody()

#define INSTANTIATE_TEST_SUITE_P(prefix, fixture, values)                                          \
  static int prefix##_##fixture##_inst = ([] {                                                     \
    static auto vals = values;                                                                     \
    for (size_t i = 0; i < vals.size(); i++)                                                       \
      for (auto& b : ::testing::internal::ParamBodies<fixture>::get()) {                          \
        auto* pv = &vals[i];                                                                       \
        auto body = b.second;                                                                      \
        ::testing::internal::registry().push_back(                                                 \
            {std::string(#prefix "/" #fixture ".") + b.first + "/" + std::to_string(i),            \
             [pv, body] { fixture::param() = pv; body(); }});                                      \
      }                                                                                            \
    return 0;                                                                                      \
  }())

#define EXPECT_EQ(a, b) \
  if (::testing::internal::eq((a), (b), #a, #b, __FILE__, __LINE__)) ; else ::testing::internal::Msg(true)
#define ASSERT_EQ(a, b) EXPECT_EQ(a, b)
#define EXPECT_TRUE(x) \
  if (::testing::internal::truth(!!(x), true, #x, __FILE__, __LINE__)) ; else ::testing::internal::Msg(true)
#define EXPECT_FALSE(x) \
  if (::testing::internal::truth(!!(x), false, #x, __FILE__, __LINE__)) ; else ::testing::internal::Msg(true)
