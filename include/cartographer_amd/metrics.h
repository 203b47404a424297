// Metrics and score histograms of the constraint-builder drop-ins.
//
// The metric interfaces follow the reference's cartographer/metrics
// (counter.h, gauge.h, histogram.h, family_factory.h): Counter, Gauge and
// Histogram with a Null() instance, labelled Family<T>, and a FamilyFactory
// that a caller (e.g. a Prometheus exporter) implements and hands to
// ConstraintBuilder{2D,3D}::RegisterMetrics. InMemoryFamilyFactory is a
// small implementation that keeps the values in memory (tests, and callers
// without an exporter).
//
// ScoreHistogram is common::Histogram (common/histogram.cc:27-75): the
// builders' score_histogram_, printed with ToString(10) when log_matches is
// on (constraint_builder_2d.cc:289-293).
#ifndef CARTOGRAPHER_AMD_METRICS_H_
#define CARTOGRAPHER_AMD_METRICS_H_

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

namespace cartographer_amd {
namespace metrics {

class Counter {
 public:
  static Counter* Null();
  virtual ~Counter() = default;
  virtual void Increment() = 0;
  virtual void Increment(double by_value) = 0;
};

class Gauge {
 public:
  static Gauge* Null();
  virtual ~Gauge() = default;
  virtual void Increment() = 0;
  virtual void Increment(double by_value) = 0;
  virtual void Decrement() = 0;
  virtual void Decrement(double by_value) = 0;
  virtual void Set(double value) = 0;
};

class Histogram {
 public:
  using BucketBoundaries = std::vector<double>;
  static Histogram* Null();
  // metrics/histogram.cc:39-62.
  static BucketBoundaries FixedWidth(double width, int num_finite_buckets) {
    BucketBoundaries b;
    double boundary = 0;
    for (int i = 0; i < num_finite_buckets; ++i) b.push_back(boundary += width);
    return b;
  }
  static BucketBoundaries ScaledPowersOf(double base, double scale_factor, double max_value) {
    BucketBoundaries b;
    if (!(base > 1) || !(scale_factor > 0)) std::abort();  // CHECK_GT
    for (double boundary = scale_factor; boundary < max_value; boundary *= base)
      b.push_back(boundary);
    return b;
  }
  virtual ~Histogram() = default;
  virtual void Observe(double value) = 0;
};

namespace internal {
struct NullCounter : Counter {
  void Increment() override {}
  void Increment(double) override {}
};
struct NullGauge : Gauge {
  void Increment() override {}
  void Increment(double) override {}
  void Decrement() override {}
  void Decrement(double) override {}
  void Set(double) override {}
};
struct NullHistogram : Histogram {
  void Observe(double) override {}
};
}  // namespace internal

inline Counter* Counter::Null() {
  static internal::NullCounter c;
  return &c;
}
inline Gauge* Gauge::Null() {
  static internal::NullGauge g;
  return &g;
}
inline Histogram* Histogram::Null() {
  static internal::NullHistogram h;
  return &h;
}

using Labels = std::map<std::string, std::string>;

template <typename MetricType>
class Family {
 public:
  static Family<MetricType>* Null();
  virtual ~Family() = default;
  virtual MetricType* Add(const Labels& labels) = 0;
};

template <typename MetricType>
class NullFamily : public Family<MetricType> {
 public:
  MetricType* Add(const Labels&) override { return MetricType::Null(); }
};

template <typename MetricType>
Family<MetricType>* Family<MetricType>::Null() {
  static NullFamily<MetricType> f;
  return &f;
}

class FamilyFactory {
 public:
  virtual ~FamilyFactory() = default;
  virtual Family<Counter>* NewCounterFamily(const std::string& name,
                                            const std::string& description) = 0;
  virtual Family<Gauge>* NewGaugeFamily(const std::string& name,
                                        const std::string& description) = 0;
  virtual Family<Histogram>* NewHistogramFamily(const std::string& name,
                                                const std::string& description,
                                                const Histogram::BucketBoundaries& boundaries) = 0;
};

// ---- in-memory implementation ------------------------------------------------
class ValueCounter : public Counter {
 public:
  void Increment() override { Increment(1.); }
  void Increment(double v) override {
    std::lock_guard<std::mutex> g(mu_);
    value_ += v;
  }
  double value() const {
    std::lock_guard<std::mutex> g(mu_);
    return value_;
  }

 private:
  mutable std::mutex mu_;
  double value_ = 0.;
};

class ValueGauge : public Gauge {
 public:
  void Increment() override { Increment(1.); }
  void Increment(double v) override { Add(v); }
  void Decrement() override { Add(-1.); }
  void Decrement(double v) override { Add(-v); }
  void Set(double v) override {
    std::lock_guard<std::mutex> g(mu_);
    value_ = v;
  }
  double value() const {
    std::lock_guard<std::mutex> g(mu_);
    return value_;
  }

 private:
  void Add(double v) {
    std::lock_guard<std::mutex> g(mu_);
    value_ += v;
  }
  mutable std::mutex mu_;
  double value_ = 0.;
};

// Prometheus semantics: bucket k counts observations <= boundaries[k] and
// above the previous boundary; the last bucket (+Inf) the rest.
class BucketHistogram : public Histogram {
 public:
  explicit BucketHistogram(BucketBoundaries b) : bounds_(std::move(b)), counts_(bounds_.size() + 1) {}
  void Observe(double v) override {
    const size_t k = std::lower_bound(bounds_.begin(), bounds_.end(), v) - bounds_.begin();
    std::lock_guard<std::mutex> g(mu_);
    ++counts_[k];
    sum_ += v;
    ++count_;
  }
  std::vector<int64_t> counts() const {
    std::lock_guard<std::mutex> g(mu_);
    return counts_;
  }
  int64_t count() const {
    std::lock_guard<std::mutex> g(mu_);
    return count_;
  }
  double sum() const {
    std::lock_guard<std::mutex> g(mu_);
    return sum_;
  }
  const BucketBoundaries& boundaries() const { return bounds_; }

 private:
  const BucketBoundaries bounds_;
  mutable std::mutex mu_;
  std::vector<int64_t> counts_;
  int64_t count_ = 0;
  double sum_ = 0.;
};

template <typename M>
class MapFamily : public Family<M> {
 public:
  explicit MapFamily(std::function<std::unique_ptr<M>()> make) : make_(std::move(make)) {}
  M* Add(const Labels& labels) override {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = metrics_[labels];
    if (!m) m = make_();
    return m.get();
  }
  // nullptr if no metric with these labels was added.
  M* Find(const Labels& labels) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = metrics_.find(labels);
    return it == metrics_.end() ? nullptr : it->second.get();
  }

 private:
  std::function<std::unique_ptr<M>()> make_;
  mutable std::mutex mu_;
  std::map<Labels, std::unique_ptr<M>> metrics_;
};

class InMemoryFamilyFactory : public FamilyFactory {
 public:
  Family<Counter>* NewCounterFamily(const std::string& name, const std::string&) override {
    return Make(&counters_, name, [] { return std::unique_ptr<Counter>(new ValueCounter); });
  }
  Family<Gauge>* NewGaugeFamily(const std::string& name, const std::string&) override {
    return Make(&gauges_, name, [] { return std::unique_ptr<Gauge>(new ValueGauge); });
  }
  Family<Histogram>* NewHistogramFamily(const std::string& name, const std::string&,
                                        const Histogram::BucketBoundaries& b) override {
    return Make(&histograms_, name, [b] { return std::unique_ptr<Histogram>(new BucketHistogram(b)); });
  }
  // Lookups for tests and exporters: nullptr if absent.
  const ValueCounter* counter(const std::string& name, const Labels& labels) const {
    return Find<ValueCounter>(counters_, name, labels);
  }
  const ValueGauge* gauge(const std::string& name, const Labels& labels = {}) const {
    return Find<ValueGauge>(gauges_, name, labels);
  }
  const BucketHistogram* histogram(const std::string& name, const Labels& labels) const {
    return Find<BucketHistogram>(histograms_, name, labels);
  }

 private:
  template <typename M>
  using Families = std::map<std::string, std::unique_ptr<MapFamily<M>>>;
  template <typename M, typename F>
  Family<M>* Make(Families<M>* fams, const std::string& name, F make) {
    std::lock_guard<std::mutex> g(mu_);
    auto& f = (*fams)[name];
    if (!f) f.reset(new MapFamily<M>(make));
    return f.get();
  }
  template <typename T, typename M>
  const T* Find(const Families<M>& fams, const std::string& name, const Labels& labels) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = fams.find(name);
    if (it == fams.end()) return nullptr;
    return static_cast<const T*>(it->second->Find(labels));
  }
  mutable std::mutex mu_;
  Families<Counter> counters_;
  Families<Gauge> gauges_;
  Families<Histogram> histograms_;
};

}  // namespace metrics

// common::Histogram (common/histogram.cc:27-75). Numbers print as absl::StrCat
// prints them: integers in decimal, floats with six significant digits (%g).
class ScoreHistogram {
 public:
  void Add(float value) { values_.push_back(value); }
  size_t size() const { return values_.size(); }

  std::string ToString(int buckets) const {
    if (buckets < 1) std::abort();  // CHECK_GE(buckets, 1)
    if (values_.empty()) return "Count: 0";
    const float min = *std::min_element(values_.begin(), values_.end());
    const float max = *std::max_element(values_.begin(), values_.end());
    const float mean = std::accumulate(values_.begin(), values_.end(), 0.f) / values_.size();
    std::string result = "Count: " + std::to_string(values_.size()) + "  Min: " + G(min) +
                         "  Max: " + G(max) + "  Mean: " + G(mean);
    if (min == max) return result;
    float lower_bound = min;
    int total_count = 0;
    for (int i = 0; i != buckets; ++i) {
      const float upper_bound =
          (i + 1 == buckets) ? max : (max * (i + 1) / buckets + min * (buckets - i - 1) / buckets);
      int count = 0;
      for (const float value : values_)
        if (lower_bound <= value && (i + 1 == buckets ? value <= upper_bound : value < upper_bound))
          ++count;
      total_count += count;
      char head[96];
      std::snprintf(head, sizeof(head), "\n[%f, %f%c", lower_bound, upper_bound,
                    i + 1 == buckets ? ']' : ')');
      result += head;
      constexpr int kMaxBarChars = 20;
      const int bar = static_cast<int>((count * kMaxBarChars + values_.size() / 2) / values_.size());
      result += "\t";
      for (int k = 0; k != kMaxBarChars; ++k) result += (k < (kMaxBarChars - bar)) ? " " : "#";
      result += "\tCount: " + std::to_string(count) + " (" + G(count * 1e2f / values_.size()) +
                "%)" + "\tTotal: " + std::to_string(total_count) + " (" +
                G(total_count * 1e2f / values_.size()) + "%)";
      lower_bound = upper_bound;
    }
    return result;
  }

 private:
  static std::string G(float v) {
    char buf[32];
    std::snprintf(buf, sizeof(buf), "%g", static_cast<double>(v));
    return buf;
  }
  std::vector<float> values_;
};

// Where the builders' log_matches lines go (LOG(INFO) in the reference). The
// default writes them to stderr only when CSM_LOG_INFO is set (glog keeps INFO
// out of the terminal by default); set_log_sink on a builder captures them.
using LogSink = std::function<void(const std::string&)>;
inline LogSink DefaultLogSink(const char* who) {
  return [who](const std::string& line) {
    static const bool on = std::getenv("CSM_LOG_INFO") != nullptr;
    if (on) std::fprintf(stderr, "I %s: %s\n", who, line.c_str());
  };
}

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_METRICS_H_
