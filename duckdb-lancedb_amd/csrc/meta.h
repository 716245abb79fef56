// Metadata columns of multi-column LANCE indexes and the predicate evaluator
// behind filtered search (internal; not public ABI).
//
// Reference (paths relative to /root/reference):
//   rust_lib/src/lance_manager.rs:62-126   create_from_arrow: the table schema is
//       `label` + the imported fields; the vector column is the first
//       FixedSizeList<Float32>, every other field is a metadata column
//   rust_lib/src/lance_manager.rs:251-301  add_batch_arrow: a struct array of
//       [vector, extra...] rows; labels assigned densely; the array is taken
//       over by the callee (release called, C++ side left released)
//   src/lance_optimizer.cpp:137-344        ExpressionToLancePredicate: the
//       Lance-SQL predicate strings pushed into the search (comparisons of a
//       column and a constant, AND / OR, NOT (..), IS [NOT] NULL, [NOT] IN (..),
//       BETWEEN as two comparisons; literals '..' with '' escapes, integers,
//       DuckDB float text, true / false, NULL)
//   src/lance_index.cpp:442-453            Search(.., predicate) -> the FFI
// Semantics: prefilter (LanceDB only_if): the top-k is taken over the live rows
// whose predicate is TRUE (SQL three-valued logic: NULL is not TRUE), which is
// what lance_optimizer_filter.test:36-44 and :57-64 need (k rows among the
// matches, not a post-filtered top-k).  The implicit `label` column (int64,
// lance_manager.rs:232-233) is always available.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

// Arrow C Data Interface (https://arrow.apache.org/docs/format/CDataInterface.html), the
// stable C ABI DuckDB's ArrowConverter produces (lance_index.cpp:297-304, :340-354)
struct ArrowSchema {
	const char *format;
	const char *name;
	const char *metadata;
	int64_t flags;
	int64_t n_children;
	struct ArrowSchema **children;
	struct ArrowSchema *dictionary;
	void (*release)(struct ArrowSchema *);
	void *private_data;
};
struct ArrowArray {
	int64_t length;
	int64_t null_count;
	int64_t offset;
	int64_t n_buffers;
	int64_t n_children;
	const void **buffers;
	struct ArrowArray **children;
	struct ArrowArray *dictionary;
	void (*release)(struct ArrowArray *);
	void *private_data;
};

namespace lhip {

enum ColType : int { COL_INT = 0, COL_FLOAT = 1, COL_BOOL = 2, COL_STRING = 3 };

// scalar index of one column (lance_detached_create_scalar_index, the call at
// lance_index.cpp:481-486; LanceDB BTREE / BITMAP): the non-NULL slots of
// [0, n_indexed) sorted by (value, slot).  Comparisons of the column with a
// literal take a binary-searched range of it instead of comparing every row;
// slots appended later are compared one by one.
struct ColIndex {
	std::string type;            // "BTREE" | "BITMAP" (same structure here)
	int64_t n_indexed = 0;
	std::vector<uint32_t> perm;  // slots sorted by value
};

// one metadata column, values per slot (slot order = ascending label order)
struct MetaColumn {
	std::string name;
	std::string arrow_format;  // as declared by the schema
	ColType type = COL_INT;
	std::vector<int64_t> i;    // COL_INT, COL_BOOL (0/1)
	std::vector<double> f;     // COL_FLOAT
	std::vector<std::string> s;  // COL_STRING
	std::vector<uint8_t> valid;  // 1 = non-NULL
	std::shared_ptr<ColIndex> index;  // scalar index, if created
	size_t size() const { return valid.size(); }
	void build_index(const std::string &type);  // over the current rows
};

struct MetaStore {
	std::string vector_name;  // name of the FixedSizeList column
	int vector_pos = 0;       // its position among the struct's children
	int dim = 0;
	std::vector<MetaColumn> cols;

	// schema of a create_from_arrow table: "+s" with one "+w:<dim>" float32 child
	static std::unique_ptr<MetaStore> from_schema(const ArrowSchema *schema);
	// a struct array of the table's columns: vectors (row-major num x dim f32)
	// out, metadata appended; returns the row count.  Does not release.
	int64_t import_batch(const ArrowSchema *schema, const ArrowArray *array, std::vector<float> &vectors);
	// compaction: keep slots `keep` (ascending)
	void keep_slots(const std::vector<int64_t> &keep);
	// append rows [from] of another store with the same columns
	void append_rows(const MetaStore &src, const std::vector<int64_t> &src_slots);
	void truncate(size_t n);
	// rows ingested through the vector-only entry points: every column NULL
	void append_nulls(int64_t n);
	// persistence: one serialized record of rows [s0, s0+n)
	void serialize_rows(int64_t s0, int64_t n, std::vector<uint8_t> &out) const;
	void deserialize_rows(const uint8_t *p, size_t len);
	void serialize_schema(std::vector<uint8_t> &out) const;
	static std::unique_ptr<MetaStore> deserialize_schema(const uint8_t *p, size_t len);
};

// Evaluates `predicate` over slots [0, n): mask[s] = 1 iff live[s] and the
// predicate is TRUE for slot s.  meta may be null (only `label` exists).
// Throws Error on a syntax error or an unknown column.  Returns the count.
int64_t eval_predicate(const std::string &predicate, const MetaStore *meta, const std::vector<int64_t> &labels,
                       const std::vector<uint8_t> &live, std::vector<uint8_t> &mask);

}  // namespace lhip
