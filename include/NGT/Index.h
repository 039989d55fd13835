/*
 * NGT/Index.h -- the C++ API of NGT 1.13.8 (NGT::Index, NGT::Property,
 * NGT::SearchContainer / NGT::SearchQuery, NGT::ObjectDistances,
 * NGT::ObjectSpace) served by the MI355X build.
 *
 * Header-only: every member is an inline call into the C ABI of
 * libngt_amd.so (include/NGT/Capi.h), so a program written against the
 * reference's C++ headers compiles against this directory, links
 * -lngt_amd, and runs its searches on the GPU -- no C++ symbols cross the
 * library boundary.  The shapes follow the reference:
 *
 *   NGT::Index           lib/NGT/Index.h:362-547 (open/create/append/insert/
 *                        createIndex/save/search/linearSearch/searchUsingOnlyGraph/
 *                        getObjectSpace/getProperty/allocateObject/...)
 *   NGT::Property        lib/NGT/Index.h:45-282, 1603-1651; Graph.h:383-524
 *   NGT::SearchContainer lib/NGT/Common.h:2007-2085 (size, radius,
 *   NGT::SearchQuery     explorationCoefficient, edgeSize, counters, results)
 *                        Common.h:2087-2114
 *   NGT::ObjectDistance  lib/NGT/Common.h:1937-1992
 *   NGT::ObjectDistances lib/NGT/ObjectSpace.h:26-91
 *   NGT::ObjectSpace     lib/NGT/ObjectSpace.h:146-292 (enums, getObject)
 *
 * Errors surface as NGT::Exception carrying the C API's message.  Entry points
 * of graph maintenance (remove, optimizer, refine) and graph-only
 * construction throw: they are outside this build's scope.
 */
#ifndef NGT_AMD_CXX_INDEX_H
#define NGT_AMD_CXX_INDEX_H

#include <sys/stat.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <sstream>
#include <string>
#include <typeinfo>
#include <utility>
#include <vector>

#include "Capi.h"

namespace NGT {

typedef float Distance;

class Exception : public std::exception {
 public:
  Exception() {}
  explicit Exception(const std::string& m) : message(m) {}
  const char* what() const noexcept override { return message.c_str(); }
  std::string& getMessage() { return message; }

 private:
  std::string message;
};

namespace detail {
// One NGTError per call: the C API writes its "Capi : <func>() : Error: ..."
// message there, which becomes the exception text.
struct Err {
  NGTError e;
  Err() : e(ngt_create_error_object()) {}
  ~Err() { ngt_destroy_error_object(e); }
  [[noreturn]] void raise(const char* where) const {
    std::string m = ngt_get_error_string(e);
    throw Exception(std::string(where) + ": " + (m.empty() ? "failed" : m));
  }
  operator NGTError() const { return e; }
};
}  // namespace detail

#pragma pack(push, 2)
class ObjectDistance {
 public:
  ObjectDistance() : id(0), distance(0.0f) {}
  ObjectDistance(unsigned int i, float d) : id(i), distance(d) {}
  bool operator==(const ObjectDistance& o) const { return distance == o.distance && id == o.id; }
  bool operator<(const ObjectDistance& o) const { return distance == o.distance ? id < o.id : distance < o.distance; }
  bool operator>(const ObjectDistance& o) const { return distance == o.distance ? id > o.id : distance > o.distance; }
  void set(unsigned int i, float d) {
    id = i;
    distance = d;
  }
  uint32_t id;
  float distance;
};
#pragma pack(pop)

class ObjectDistances : public std::vector<ObjectDistance> {};

// An allocated query (Index::allocateObject): the caller's values as floats
// of the object dimension; the device converts them to the object type and
// normalizes them for the normalized metrics, as Index::allocateObject does.
class Object {
 public:
  std::vector<float> values;
  float& operator[](size_t i) { return values[i]; }
};

class ObjectSpace {
 public:
  enum DistanceType {
    DistanceTypeNone = -1,
    DistanceTypeL1 = 0,
    DistanceTypeL2 = 1,
    DistanceTypeHamming = 2,
    DistanceTypeAngle = 3,
    DistanceTypeCosine = 4,
    DistanceTypeNormalizedAngle = 5,
    DistanceTypeNormalizedCosine = 6,
    DistanceTypeJaccard = 7,
    DistanceTypeSparseJaccard = 8,
    DistanceTypeNormalizedL2 = 9,
    DistanceTypePoincare = 100,
    DistanceTypeLorentz = 101
  };
  enum ObjectType { ObjectTypeNone = 0, Uint8 = 1, Float = 2 };

  // Borrowed pointer into the index's host mirror of object `id` (float* or
  // uint8_t* by object type), valid until the index closes (Capi.cpp:750-781).
  void* getObject(ObjectID id) {
    detail::Err err;
    void* p = objectType == Float ? static_cast<void*>(ngt_get_object_as_float(space, id, err))
                                  : static_cast<void*>(ngt_get_object_as_integer(space, id, err));
    if (p == nullptr) err.raise("NGT::ObjectSpace::getObject");
    return p;
  }
  void getObject(ObjectID id, std::vector<float>& v) {
    v.resize(dimension);
    if (objectType == Float) {
      const float* p = static_cast<const float*>(getObject(id));
      v.assign(p, p + dimension);
    } else {
      const uint8_t* p = static_cast<const uint8_t*>(getObject(id));
      for (size_t i = 0; i < dimension; i++) v[i] = p[i];
    }
  }
  size_t getDimension() const { return dimension; }
  size_t getPaddedDimension() const { return ((dimension - 1) / 16 + 1) * 16; }
  DistanceType getDistanceType() const { return distanceType; }
  ObjectType getObjectType() const { return objectType; }
  size_t getSizeOfElement() const { return objectType == Float ? 4 : 1; }

 private:
  friend class Index;
  NGTObjectSpace space = nullptr;
  size_t dimension = 0;
  DistanceType distanceType = DistanceTypeNone;
  ObjectType objectType = ObjectTypeNone;
};

class SearchContainer {
 public:
  SearchContainer() : object(nullptr) { initialize(); }
  explicit SearchContainer(Object& f) : object(&f) { initialize(); }
  SearchContainer(Object& f, ObjectID) : object(&f) { initialize(); }
  virtual ~SearchContainer() {}
  virtual void initialize() {
    size = 10;
    radius = FLT_MAX;
    explorationCoefficient = 1.1f;
    edgeSize = -1;  // -1: the index property; 0: all edges; -2: dynamic
    useAllNodesInLeaf = false;
    expectedAccuracy = -1.0f;
    distanceComputationCount = 0;
    visitCount = 0;
    result = nullptr;
  }
  void setSize(size_t s) { size = s; }
  void setResults(ObjectDistances* r) { result = r; }
  void setRadius(Distance r) { radius = r; }
  void setEpsilon(float e) { explorationCoefficient = e + 1.0; }
  void setEdgeSize(int e) { edgeSize = e; }
  void setExpectedAccuracy(float a) { expectedAccuracy = a; }
  bool resultIsAvailable() { return result != nullptr; }
  ObjectDistances& getResult() {
    if (result == nullptr) throw Exception("Inner error: results is not set");
    return *result;
  }
  Object* getObject() { return object; }

  size_t size;
  Distance radius;
  float explorationCoefficient;
  int edgeSize;
  size_t distanceComputationCount;
  bool useAllNodesInLeaf;
  size_t visitCount;
  float expectedAccuracy;

 protected:
  Object* object;
  ObjectDistances* result;
};

// NGT::QueryContainer: the query kept as the caller's float / double / uint8_t
// vector (Common.h:2087-2110).
class QueryContainer {
 public:
  template <typename QTYPE>
  explicit QueryContainer(const std::vector<QTYPE>& q) {
    setQuery(q);
  }
  template <typename QTYPE>
  void setQuery(const std::vector<QTYPE>& q) {
    if (typeid(QTYPE) != typeid(float) && typeid(QTYPE) != typeid(double) && typeid(QTYPE) != typeid(uint8_t))
      throw Exception("NGT::SearchQuery: Invalid query type!");
    query.assign(q.begin(), q.end());
    queryType = &typeid(QTYPE);
  }
  const std::vector<float>& getQueryValues() const { return query; }
  const std::type_info& getQueryType() const { return *queryType; }

 private:
  std::vector<float> query;
  const std::type_info* queryType = &typeid(float);
};

class SearchQuery : public QueryContainer, public SearchContainer {
 public:
  template <typename QTYPE>
  explicit SearchQuery(const std::vector<QTYPE>& q) : QueryContainer(q) {}
};

class NeighborhoodGraph {
 public:
  enum GraphType {
    GraphTypeNone = 0,
    GraphTypeANNG = 1,
    GraphTypeKNNG = 2,
    GraphTypeBKNNG = 3,
    GraphTypeONNG = 4,
    GraphTypeIANNG = 5,
    GraphTypeDNNG = 6
  };
  enum SeedType {
    SeedTypeNone = 0,
    SeedTypeRandomNodes = 1,
    SeedTypeFixedNodes = 2,
    SeedTypeFirstNode = 3,
    SeedTypeAllLeafNodes = 4
  };
  // NeighborhoodGraph::Property (Graph.h:383-524): the graph half of NGT::Property
  class Property {
   public:
    Property() { setDefault(); }
    void setDefault() {
      truncationThreshold = 0;
      edgeSizeForCreation = 10;
      edgeSizeForSearch = 0;
      edgeSizeLimitForCreation = 5;
      insertionRadiusCoefficient = 1.1;
      seedSize = 10;
      seedType = SeedTypeNone;
      truncationThreadPoolSize = 8;
      batchSizeForCreation = 200;
      graphType = GraphTypeANNG;
      dynamicEdgeSizeBase = 30;
      dynamicEdgeSizeRate = 20;
      buildTimeLimit = 0.0;
      outgoingEdge = 10;
      incomingEdge = 80;
    }
    int16_t truncationThreshold;
    int16_t edgeSizeForCreation;
    int16_t edgeSizeForSearch;
    int16_t edgeSizeLimitForCreation;
    double insertionRadiusCoefficient;
    int16_t seedSize;
    SeedType seedType;
    int16_t truncationThreadPoolSize;
    int16_t batchSizeForCreation;
    GraphType graphType;
    int16_t dynamicEdgeSizeBase;
    int16_t dynamicEdgeSizeRate;
    float buildTimeLimit;
    int16_t outgoingEdge;
    int16_t incomingEdge;
  };
};

class Property;

class Index {
 public:
  // Index::Property (Index.h:45-282): the index half of NGT::Property
  class Property {
   public:
    typedef ObjectSpace::ObjectType ObjectType;
    typedef ObjectSpace::DistanceType DistanceType;
    typedef NeighborhoodGraph::SeedType SeedType;
    typedef NeighborhoodGraph::GraphType GraphType;
    enum ObjectAlignment { ObjectAlignmentNone = 0, ObjectAlignmentTrue = 1, ObjectAlignmentFalse = 2 };
    enum IndexType { IndexTypeNone = 0, GraphAndTree = 1, Graph = 2 };
    enum DatabaseType { DatabaseTypeNone = 0, Memory = 1, MemoryMappedFile = 2 };
    Property() { setDefault(); }
    void setDefault() {
      dimension = 0;
      threadPoolSize = 32;
      objectType = ObjectSpace::Float;
      distanceType = ObjectSpace::DistanceTypeL2;
      indexType = GraphAndTree;
      objectAlignment = ObjectAlignmentFalse;
      pathAdjustmentInterval = 0;
      databaseType = Memory;
      prefetchOffset = 0;
      prefetchSize = 0;
      accuracyTable = "";
    }
    int dimension;
    int threadPoolSize;
    ObjectType objectType;
    DistanceType distanceType;
    IndexType indexType;
    DatabaseType databaseType;
    ObjectAlignment objectAlignment;
    int pathAdjustmentInterval;
    int prefetchOffset;
    int prefetchSize;
    std::string accuracyTable;
  };

  Index() {}
  explicit Index(NGT::Property& prop);
  Index(const std::string& database, bool rdOnly = false) { open(database, rdOnly); }
  virtual ~Index() { close(); }

  void open(const std::string& database, bool rdOnly = false) {
    close();
    detail::Err err;
    index = ngt_open_index(database.c_str(), err);
    if (index == nullptr) err.raise("NGT::Index::open");
    path = database;
    readOnly = rdOnly;
    loadSpace();
  }
  void close() {
    if (index) ngt_close_index(index);
    index = nullptr;
    path.clear();
  }
  void save() {
    if (path.empty()) throw Exception("NGT::Index::saveIndex: path is empty");
    saveIndex(path);
  }
  void save(std::string indexPath) { saveIndex(indexPath); }
  virtual void saveIndex(const std::string& ofile) {
    detail::Err err;
    if (!ngt_save_index(handle(), ofile.c_str(), err)) err.raise("NGT::Index::saveIndex");
  }

  static void mkdir(const std::string& dir) {
    if (::mkdir(dir.c_str(), S_IRWXU | S_IRGRP | S_IXGRP | S_IROTH | S_IXOTH) != 0)
      throw Exception("NGT::Index::mkdir: Cannot make the specified directory. " + dir);
  }
  // an empty GraphAndTree index directory (Index.cpp:113-139)
  static void create(const std::string& database, NGT::Property& prop, bool redirect = false) {
    createGraphAndTree(database, prop, redirect);
  }
  static void createGraphAndTree(const std::string& database, NGT::Property& prop, bool redirect = false);
  static void createGraph(const std::string&, NGT::Property&, const std::string& = "", size_t = 0, bool = false) {
    throw Exception("NGT::Index::createGraph: graph-only construction is not part of this build");
  }

  // Index::append / insert (Index.h:1655-1678): the object joins the
  // repository (normalized for the normalized metrics); createIndex builds
  // its graph node.  Returns the object id.
  template <typename T>
  size_t append(const std::vector<T>& object) {
    std::vector<float> v(object.begin(), object.end());
    detail::Err err;
    ObjectID id = ngt_append_index_as_float(handle(), v.data(), (uint32_t)v.size(), err);
    if (id == 0) err.raise("NGT::Index::append");
    return id;
  }
  template <typename T>
  size_t insert(const std::vector<T>& object) {
    return append(object);
  }
  virtual void append(const float* data, size_t dataSize) {
    for (size_t i = 0; i < dataSize; i++)
      append(std::vector<float>(data + i * space.getDimension(), data + (i + 1) * space.getDimension()));
  }
  virtual void append(const double* data, size_t dataSize) {
    for (size_t i = 0; i < dataSize; i++)
      append(std::vector<double>(data + i * space.getDimension(), data + (i + 1) * space.getDimension()));
  }
  // GraphAndTreeIndex::createIndex (Index.cpp:1158-1257) on the device
  virtual void createIndex(size_t threadNumber, size_t sizeOfRepository = 0) {
    (void)sizeOfRepository;
    detail::Err err;
    if (!ngt_create_index(handle(), (uint32_t)threadNumber, err)) err.raise("NGT::Index::createIndex");
  }
  virtual size_t getObjectRepositorySize() {
    detail::Err err;
    return ngt_get_object_repository_size(handle(), err);
  }

  // Index::allocateObject (Index.h:437-441) -- a query object
  virtual Object* allocateObject(const std::vector<double>& obj) { return makeObject(obj); }
  virtual Object* allocateObject(const std::vector<float>& obj) { return makeObject(obj); }
  virtual Object* allocateObject(const std::vector<uint8_t>& obj) { return makeObject(obj); }
  virtual Object* allocateObject(const float* obj, size_t size) {
    return makeObject(std::vector<float>(obj, obj + size));
  }
  virtual void deleteObject(Object* po) { delete po; }
  virtual size_t getSizeOfElement() { return space.getSizeOfElement(); }

  virtual void getProperty(NGT::Property& prop);
  virtual void setProperty(NGT::Property&) {
    throw Exception("NGT::Index::setProperty: properties are fixed once the index is open in this build");
  }

  // GraphAndTreeIndex::search (Index.h:1570-1577) / GraphIndex::search: tree
  // seeds for GraphAndTree indexes, getRandomSeeds for graph-only ones
  virtual void search(SearchContainer& sc) {
    if (sc.getObject() == nullptr) throw Exception("NGT::Index::search: the search container has no object");
    searchValues(sc, sc.getObject()->values, false);
  }
  virtual void search(SearchQuery& sq) { searchValues(sq, sq.getQueryValues(), false); }
  // Index::searchUsingOnlyGraph (Index.h:479-484): random seeds, no tree
  void searchUsingOnlyGraph(SearchContainer& sc) {
    if (sc.getObject() == nullptr) throw Exception("NGT::Index::search: the search container has no object");
    searchValues(sc, sc.getObject()->values, true);
  }
  void searchUsingOnlyGraph(SearchQuery& sq) { searchValues(sq, sq.getQueryValues(), true); }
  // Index::linearSearch (Index.h:453-454, GraphIndex::linearSearch Index.h:729-749)
  virtual void linearSearch(SearchContainer& sc) {
    if (sc.getObject() == nullptr) throw Exception("NGT::Index::linearSearch: no object");
    linearValues(sc, sc.getObject()->values);
  }
  virtual void linearSearch(SearchQuery& sq) { linearValues(sq, sq.getQueryValues()); }

  // Batched device search (extension): queries [nq][dimension] row-major;
  // results[i] receives query i's neighbours.
  void batchSearch(const std::vector<float>& queries, size_t nq, size_t size, float epsilon,
                   std::vector<ObjectDistances>& results, float radius = FLT_MAX, int edgeSize = -1) {
    const size_t dim = space.getDimension() + (space.getDistanceType() == ObjectSpace::DistanceTypeSparseJaccard);
    if (queries.size() != nq * dim) throw Exception("NGT::Index::batchSearch: queries are not [nq][dimension]");
    std::vector<uint32_t> ids(nq * size), n(nq);
    std::vector<float> ds(nq * size);
    detail::Err err;
    if (!ngt_batch_search_index(handle(), queries.data(), (uint32_t)nq, (int32_t)dim, size, epsilon, radius,
                                edgeSize, ids.data(), ds.data(), n.data(), err))
      err.raise("NGT::Index::batchSearch");
    results.resize(nq);
    for (size_t q = 0; q < nq; q++) {
      results[q].clear();
      for (uint32_t j = 0; j < n[q]; j++) results[q].push_back(ObjectDistance(ids[q * size + j], ds[q * size + j]));
    }
  }

  virtual void remove(ObjectID id, bool force = false) {
    (void)force;
    detail::Err err;
    if (!ngt_remove_index(handle(), id, err)) err.raise("NGT::Index::remove");
  }
  virtual ObjectSpace& getObjectSpace() { return space; }
  // GraphIndex::getEpsilonFromExpectedAccuracy over the prf AccuracyTable
  // (Index.h:293-360, AccuracyTable::getEpsilon)
  float getEpsilonFromExpectedAccuracy(double accuracy);
  std::vector<float> makeSparseObject(std::vector<uint32_t>& object) {
    if (space.getDistanceType() != ObjectSpace::DistanceTypeSparseJaccard)
      throw Exception("NGT::Index::makeSparseObject: Not sparse jaccard.");
    std::vector<float> obj(std::max(space.getDimension() + 1, object.size() + 1), 0.0f);
    for (size_t i = 0; i < object.size(); i++) memcpy(&obj[i], &object[i], sizeof(float));
    return obj;
  }
  std::string getPath() { return path; }
  void enableLog() {}
  void disableLog() {}
  NGTIndex getHandle() { return handle(); }

 protected:
  NGTIndex handle() {
    if (index == nullptr) throw Exception("NGT::Index::getIndex: Index is unavailable.");
    return index;
  }
  template <typename T>
  Object* makeObject(const std::vector<T>& obj) {
    Object* o = new Object();
    o->values.assign(obj.begin(), obj.end());
    return o;
  }
  void loadSpace();
  void searchValues(SearchContainer& sc, const std::vector<float>& q, bool graphOnly);
  void linearValues(SearchContainer& sc, const std::vector<float>& q);

  NGTIndex index = nullptr;
  std::string path;
  bool readOnly = false;
  ObjectSpace space;
};

// NGT::Property = Index::Property + NeighborhoodGraph::Property (Index.h:1603-1651)
class Property : public Index::Property, public NeighborhoodGraph::Property {
 public:
  void setDefault() {
    Index::Property::setDefault();
    NeighborhoodGraph::Property::setDefault();
  }
  // load from / save to <index>/prf (PropertySet keys, Common.h:573-666)
  void load(const std::string& database) {
    detail::Err err;
    NGTIndex ix = ngt_open_index(database.c_str(), err);
    if (ix == nullptr) err.raise("NGT::Property::load");
    NGTProperty p = ngt_create_property(err);
    ngt_get_property(ix, p, err);
    fromCapi(p);
    ngt_destroy_property(p);
    ngt_close_index(ix);
  }

  // field <-> prf key (Index.h:105-261, Graph.h:423-489)
  NGTProperty toCapi() const {
    detail::Err err;
    NGTProperty p = ngt_create_property(err);
    if (p == nullptr) err.raise("NGT::Property");
    auto set = [&](const char* k, const std::string& v) { ngt_set_property_value(p, k, v.c_str(), err); };
    auto num = [](double v) {
      std::ostringstream os;
      os << v;
      return os.str();
    };
    set("Dimension", std::to_string(dimension));
    set("ObjectType", objectType == ObjectSpace::Uint8 ? "Integer-1" : "Float-4");
    set("DistanceType", distanceName(distanceType));
    set("IndexType", indexType == Graph ? "Graph" : "GraphAndTree");
    set("ThreadPoolSize", std::to_string(threadPoolSize));
    set("PathAdjustmentInterval", std::to_string(pathAdjustmentInterval));
    if (prefetchOffset) set("PrefetchOffset", std::to_string(prefetchOffset));
    if (prefetchSize) set("PrefetchSize", std::to_string(prefetchSize));
    if (!accuracyTable.empty()) set("AccuracyTable", accuracyTable);
    set("EdgeSizeForCreation", std::to_string(edgeSizeForCreation));
    set("EdgeSizeForSearch", std::to_string(edgeSizeForSearch));
    set("EdgeSizeLimitForCreation", std::to_string(edgeSizeLimitForCreation));
    set("EpsilonForCreation", num(insertionRadiusCoefficient - 1.0));
    set("SeedSize", std::to_string(seedSize));
    static const char* seeds[] = {"None", "RandomNodes", "FixedNodes", "FirstNode", "AllLeafNodes"};
    set("SeedType", seeds[seedType >= 0 && seedType < 5 ? seedType : 0]);
    set("TruncationThreadPoolSize", std::to_string(truncationThreadPoolSize));
    set("BatchSizeForCreation", std::to_string(batchSizeForCreation));
    static const char* graphs[] = {"None", "ANNG", "KNNG", "BKNNG", "ONNG", "IANNG", "DNNG"};
    set("GraphType", graphs[graphType >= 0 && graphType < 7 ? graphType : 1]);
    set("DynamicEdgeSizeBase", std::to_string(dynamicEdgeSizeBase));
    set("DynamicEdgeSizeRate", std::to_string(dynamicEdgeSizeRate));
    set("BuildTimeLimit", num(buildTimeLimit));
    set("OutgoingEdge", std::to_string(outgoingEdge));
    set("IncomingEdge", std::to_string(incomingEdge));
    return p;
  }
  void fromCapi(NGTProperty p) {
    auto get = [&](const char* k) {
      detail::Err err;
      char buf[4096] = {0};
      return ngt_get_property_value(p, k, buf, sizeof buf, err) < 0 ? std::string() : std::string(buf);
    };
    auto num = [&](const char* k, double dflt) {
      std::string v = get(k);
      return v.empty() ? dflt : atof(v.c_str());
    };
    dimension = (int)num("Dimension", 0);
    objectType = get("ObjectType") == "Integer-1" ? ObjectSpace::Uint8 : ObjectSpace::Float;
    distanceType = distanceOf(get("DistanceType"));
    indexType = get("IndexType") == "Graph" ? Graph : GraphAndTree;
    threadPoolSize = (int)num("ThreadPoolSize", threadPoolSize);
    pathAdjustmentInterval = (int)num("PathAdjustmentInterval", 0);
    prefetchOffset = (int)num("PrefetchOffset", 0);
    prefetchSize = (int)num("PrefetchSize", 0);
    accuracyTable = get("AccuracyTable");
    edgeSizeForCreation = (int16_t)num("EdgeSizeForCreation", edgeSizeForCreation);
    edgeSizeForSearch = (int16_t)num("EdgeSizeForSearch", edgeSizeForSearch);
    edgeSizeLimitForCreation = (int16_t)num("EdgeSizeLimitForCreation", edgeSizeLimitForCreation);
    insertionRadiusCoefficient = num("EpsilonForCreation", insertionRadiusCoefficient - 1.0) + 1.0;
    seedSize = (int16_t)num("SeedSize", seedSize);
    const std::string st = get("SeedType");
    static const char* seeds[] = {"None", "RandomNodes", "FixedNodes", "FirstNode", "AllLeafNodes"};
    for (int i = 0; i < 5; i++)
      if (st == seeds[i]) seedType = (SeedType)i;
    truncationThreadPoolSize = (int16_t)num("TruncationThreadPoolSize", truncationThreadPoolSize);
    batchSizeForCreation = (int16_t)num("BatchSizeForCreation", batchSizeForCreation);
    const std::string gt = get("GraphType");
    static const char* graphs[] = {"None", "ANNG", "KNNG", "BKNNG", "ONNG", "IANNG", "DNNG"};
    for (int i = 0; i < 7; i++)
      if (gt == graphs[i]) graphType = (GraphType)i;
    dynamicEdgeSizeBase = (int16_t)num("DynamicEdgeSizeBase", dynamicEdgeSizeBase);
    dynamicEdgeSizeRate = (int16_t)num("DynamicEdgeSizeRate", dynamicEdgeSizeRate);
    buildTimeLimit = (float)num("BuildTimeLimit", buildTimeLimit);
    outgoingEdge = (int16_t)num("OutgoingEdge", outgoingEdge);
    incomingEdge = (int16_t)num("IncomingEdge", incomingEdge);
  }
  static const char* distanceName(ObjectSpace::DistanceType d) {
    switch (d) {
      case ObjectSpace::DistanceTypeL1: return "L1";
      case ObjectSpace::DistanceTypeHamming: return "Hamming";
      case ObjectSpace::DistanceTypeAngle: return "Angle";
      case ObjectSpace::DistanceTypeCosine: return "Cosine";
      case ObjectSpace::DistanceTypeNormalizedAngle: return "NormalizedAngle";
      case ObjectSpace::DistanceTypeNormalizedCosine: return "NormalizedCosine";
      case ObjectSpace::DistanceTypeJaccard: return "Jaccard";
      case ObjectSpace::DistanceTypeSparseJaccard: return "SparseJaccard";
      case ObjectSpace::DistanceTypeNormalizedL2: return "NormalizedL2";
      case ObjectSpace::DistanceTypePoincare: return "Poincare";
      case ObjectSpace::DistanceTypeLorentz: return "Lorentz";
      default: return "L2";
    }
  }
  static ObjectSpace::DistanceType distanceOf(const std::string& s) {
    static const ObjectSpace::DistanceType all[] = {
        ObjectSpace::DistanceTypeL1,          ObjectSpace::DistanceTypeL2,
        ObjectSpace::DistanceTypeHamming,     ObjectSpace::DistanceTypeAngle,
        ObjectSpace::DistanceTypeCosine,      ObjectSpace::DistanceTypeNormalizedAngle,
        ObjectSpace::DistanceTypeNormalizedCosine, ObjectSpace::DistanceTypeJaccard,
        ObjectSpace::DistanceTypeSparseJaccard, ObjectSpace::DistanceTypeNormalizedL2,
        ObjectSpace::DistanceTypePoincare,    ObjectSpace::DistanceTypeLorentz};
    for (auto d : all)
      if (s == distanceName(d)) return d;
    return ObjectSpace::DistanceTypeL2;
  }
};

// ---- out-of-class members (need the complete NGT::Property) ---------------
inline Index::Index(NGT::Property& prop) {
  NGTProperty p = prop.toCapi();
  detail::Err err;
  index = ngt_create_graph_and_tree_in_memory(p, err);
  ngt_destroy_property(p);
  if (index == nullptr) err.raise("NGT::Index::Index");
  loadSpace();
}

inline void Index::createGraphAndTree(const std::string& database, NGT::Property& prop, bool) {
  NGTProperty p = prop.toCapi();
  detail::Err err;
  NGTIndex ix = ngt_create_graph_and_tree(database.c_str(), p, err);
  ngt_destroy_property(p);
  if (ix == nullptr) err.raise("NGT::Index::createGraphAndTree");
  ngt_close_index(ix);
}

inline void Index::getProperty(NGT::Property& prop) {
  detail::Err err;
  NGTProperty p = ngt_create_property(err);
  if (!ngt_get_property(handle(), p, err)) {
    ngt_destroy_property(p);
    err.raise("NGT::Index::getProperty");
  }
  prop.fromCapi(p);
  ngt_destroy_property(p);
}

inline void Index::loadSpace() {
  NGT::Property prop;
  getProperty(prop);
  detail::Err err;
  space.space = ngt_get_object_space(handle(), err);
  space.dimension = (size_t)prop.dimension;
  space.distanceType = prop.distanceType;
  space.objectType = prop.objectType;
}

inline float Index::getEpsilonFromExpectedAccuracy(double accuracy) {
  NGT::Property prop;
  getProperty(prop);
  std::vector<std::pair<float, double>> table;
  std::stringstream ss(prop.accuracyTable);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    const size_t c = tok.find(':');
    if (c == std::string::npos) throw Exception("AccuracyTable: Invalid accuracy table string " + tok);
    table.push_back(std::make_pair((float)atof(tok.substr(0, c).c_str()), atof(tok.substr(c + 1).c_str())));
  }
  if (table.size() <= 2) {
    std::ostringstream m;
    m << "AccuracyTable: The accuracy table is not set yet. The table size=" << table.size();
    throw Exception(m.str());
  }
  if (accuracy > 1.0) accuracy = 1.0;
  size_t i = 0;
  while (i < table.size() && table[i].second < accuracy) i++;
  if (i == table.size()) i -= 2;
  else if (i != 0) i--;
  const std::pair<float, double> lower = table[i], upper = table[i + 1];
  float e = lower.first + (upper.first - lower.first) * (accuracy - lower.second) / (upper.second - lower.second);
  return e < -0.9f ? -0.9f : e;
}

inline void Index::searchValues(SearchContainer& sc, const std::vector<float>& q, bool graphOnly) {
  ObjectDistances& out = sc.getResult();
  out.clear();
  sc.distanceComputationCount = 0;
  sc.visitCount = 0;
  if (sc.expectedAccuracy > 0.0f) sc.setEpsilon(getEpsilonFromExpectedAccuracy(sc.expectedAccuracy));
  const float epsilon = (float)((double)sc.explorationCoefficient - 1.0);
  detail::Err err;
  if (!graphOnly) {
    NGTQuery query;
    std::vector<float> v(q);
    query.query = v.data();
    query.size = sc.size;
    query.epsilon = epsilon;
    query.accuracy = 0.0f;
    query.radius = sc.radius;
    query.edge_size = (size_t)(int64_t)sc.edgeSize;
    NGTObjectDistances r = ngt_create_empty_results(err);
    if (!ngt_search_index_with_query(handle(), query, r, err)) {
      ngt_destroy_results(r);
      err.raise("NGT::Index::search");
    }
    const uint32_t n = ngt_get_result_size(r, err);
    for (uint32_t i = 0; i < n; i++) {
      NGTObjectDistance d = ngt_get_result(r, i, err);
      out.push_back(ObjectDistance(d.id, d.distance));
    }
    ngt_destroy_results(r);
  } else {
    std::vector<uint32_t> ids(sc.size ? sc.size : 1), n(1);
    std::vector<float> ds(ids.size());
    if (!ngt_batch_search_index_using_only_graph(handle(), q.data(), 1, (int32_t)q.size(), sc.size, epsilon,
                                                 sc.radius, sc.edgeSize, ids.data(), ds.data(), n.data(), err))
      err.raise("NGT::Index::searchUsingOnlyGraph");
    for (uint32_t i = 0; i < n[0]; i++) out.push_back(ObjectDistance(ids[i], ds[i]));
  }
  uint64_t c[3] = {0, 0, 0};
  if (ngt_get_last_search_counters(handle(), c, err)) {
    sc.distanceComputationCount = (size_t)c[0];
    sc.visitCount = (size_t)c[1];
  }
}

inline void Index::linearValues(SearchContainer& sc, const std::vector<float>& q) {
  ObjectDistances& out = sc.getResult();
  out.clear();
  std::vector<uint32_t> ids(sc.size ? sc.size : 1), n(1);
  std::vector<float> ds(ids.size());
  detail::Err err;
  if (sc.size == 0) return;
  if (!ngt_batch_linear_search_index_with_radius(handle(), q.data(), 1, (int32_t)q.size(), sc.size, sc.radius,
                                                 ids.data(), ds.data(), n.data(), err))
    err.raise("NGT::Index::linearSearch");
  for (uint32_t i = 0; i < n[0]; i++) out.push_back(ObjectDistance(ids[i], ds[i]));
}

}  // namespace NGT

#endif
