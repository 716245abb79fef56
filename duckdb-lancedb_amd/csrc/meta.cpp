// Metadata columns (Arrow C Data Interface import) and the Lance-SQL predicate
// evaluator of filtered search.  Contract and reference lines: meta.h.
#include "meta.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "index.h"

namespace lhip {

// ---------------------------------------------------------------------------
// Arrow import
// ---------------------------------------------------------------------------
static bool is_fixed_f32_list(const ArrowSchema *c, int &dim) {
	if (!c || !c->format || strncmp(c->format, "+w:", 3) != 0) return false;
	if (c->n_children != 1 || !c->children[0] || !c->children[0]->format || strcmp(c->children[0]->format, "f") != 0)
		return false;
	dim = atoi(c->format + 3);
	return dim > 0;
}

static ColType col_type_of(const char *fmt) {
	const std::string f = fmt ? fmt : "";
	if (f == "c" || f == "s" || f == "i" || f == "l" || f == "C" || f == "S" || f == "I" || f == "L") return COL_INT;
	if (f == "f" || f == "g") return COL_FLOAT;
	if (f == "b") return COL_BOOL;
	if (f == "u" || f == "U") return COL_STRING;
	throw Error("unsupported Arrow column format '" + f + "' (supported: integers, float, double, boolean, utf8)");
}

std::unique_ptr<MetaStore> MetaStore::from_schema(const ArrowSchema *schema) {
	if (!schema || !schema->format || strcmp(schema->format, "+s") != 0)
		throw Error("Arrow schema must be a struct (+s) of the table's columns");
	auto m = std::make_unique<MetaStore>();
	m->vector_pos = -1;
	for (int64_t i = 0; i < schema->n_children; ++i) {
		const ArrowSchema *c = schema->children[i];
		int d = 0;
		if (m->vector_pos < 0 && is_fixed_f32_list(c, d)) {
			m->vector_pos = (int)i;
			m->dim = d;
			m->vector_name = c->name ? c->name : "vector";
			continue;
		}
		MetaColumn col;
		col.name = c && c->name ? c->name : ("col" + std::to_string(i));
		col.arrow_format = c && c->format ? c->format : "";
		col.type = col_type_of(c ? c->format : nullptr);
		if (col.name == "label") throw Error("column name 'label' is reserved (lance_manager.rs:101)");
		m->cols.push_back(std::move(col));
	}
	if (m->vector_pos < 0) throw Error("no FixedSizeList column found in schema");
	return m;
}

static inline bool bit(const void *buf, int64_t i) {
	return (static_cast<const uint8_t *>(buf)[i >> 3] >> (i & 7)) & 1;
}

int64_t MetaStore::import_batch(const ArrowSchema *schema, const ArrowArray *array, std::vector<float> &vectors) {
	if (!schema || !array) throw Error("null arrow schema/array");
	if (!schema->format || strcmp(schema->format, "+s") != 0) throw Error("Arrow batch must be a struct array (+s)");
	if (schema->n_children != (int64_t)cols.size() + 1 || array->n_children != schema->n_children)
		throw Error("Arrow batch has " + std::to_string(array->n_children) + " columns, the table " +
		            std::to_string(cols.size() + 1));
	const int64_t n = array->length, off0 = array->offset;
	int ci = 0;
	for (int64_t c = 0; c < schema->n_children; ++c) {
		const ArrowSchema *cs = schema->children[c];
		const ArrowArray *ca = array->children[c];
		if (!cs || !ca) throw Error("null Arrow child");
		const int64_t off = off0 + ca->offset;
		if (c == vector_pos) {
			int d = 0;
			if (!is_fixed_f32_list(cs, d) || d != dim)
				throw Error("vector column must be FixedSizeList<float32>[" + std::to_string(dim) + "]");
			if (ca->null_count > 0 && ca->buffers[0])
				for (int64_t r = 0; r < n; ++r)
					if (!bit(ca->buffers[0], off + r)) throw Error("NULL vector in row " + std::to_string(r));
			const ArrowArray *vals = ca->children[0];
			const float *v = static_cast<const float *>(vals->buffers[1]) + vals->offset + off * dim;
			vectors.assign(v, v + (size_t)n * dim);
			continue;
		}
		MetaColumn &col = cols[(size_t)ci++];
		if (col_type_of(cs->format) != col.type || col.arrow_format != cs->format)
			throw Error("column '" + col.name + "' has Arrow format '" + cs->format + "', the table '" +
			            col.arrow_format + "'");
		const void *vb = ca->n_buffers > 0 ? ca->buffers[0] : nullptr;
		const size_t base = col.size();
		col.valid.resize(base + (size_t)n);
		for (int64_t r = 0; r < n; ++r) col.valid[base + (size_t)r] = (!vb || ca->null_count == 0) ? 1 : bit(vb, off + r);
		const std::string f = cs->format;
		switch (col.type) {
		case COL_INT: {
			col.i.resize(base + (size_t)n);
			const void *d = ca->buffers[1];
			for (int64_t r = 0; r < n; ++r) {
				const int64_t k = off + r;
				int64_t x;
				if (f == "c") x = static_cast<const int8_t *>(d)[k];
				else if (f == "s") x = static_cast<const int16_t *>(d)[k];
				else if (f == "i") x = static_cast<const int32_t *>(d)[k];
				else if (f == "l") x = static_cast<const int64_t *>(d)[k];
				else if (f == "C") x = static_cast<const uint8_t *>(d)[k];
				else if (f == "S") x = static_cast<const uint16_t *>(d)[k];
				else if (f == "I") x = static_cast<const uint32_t *>(d)[k];
				else x = (int64_t) static_cast<const uint64_t *>(d)[k];
				col.i[base + (size_t)r] = col.valid[base + (size_t)r] ? x : 0;
			}
			break;
		}
		case COL_FLOAT: {
			col.f.resize(base + (size_t)n);
			for (int64_t r = 0; r < n; ++r) {
				const int64_t k = off + r;
				const double x = f == "f" ? (double) static_cast<const float *>(ca->buffers[1])[k]
				                          : static_cast<const double *>(ca->buffers[1])[k];
				col.f[base + (size_t)r] = col.valid[base + (size_t)r] ? x : 0.0;
			}
			break;
		}
		case COL_BOOL: {
			col.i.resize(base + (size_t)n);
			for (int64_t r = 0; r < n; ++r)
				col.i[base + (size_t)r] = col.valid[base + (size_t)r] ? (int64_t)bit(ca->buffers[1], off + r) : 0;
			break;
		}
		case COL_STRING: {
			col.s.resize(base + (size_t)n);
			const char *data = static_cast<const char *>(ca->buffers[2]);
			for (int64_t r = 0; r < n; ++r) {
				if (!col.valid[base + (size_t)r]) continue;
				const int64_t k = off + r;
				int64_t a, b;
				if (f == "u") {
					a = static_cast<const int32_t *>(ca->buffers[1])[k];
					b = static_cast<const int32_t *>(ca->buffers[1])[k + 1];
				} else {
					a = static_cast<const int64_t *>(ca->buffers[1])[k];
					b = static_cast<const int64_t *>(ca->buffers[1])[k + 1];
				}
				col.s[base + (size_t)r].assign(data + a, (size_t)(b - a));
			}
			break;
		}
		}
	}
	return n;
}

void MetaStore::keep_slots(const std::vector<int64_t> &keep) {
	for (auto &c : cols) {
		MetaColumn nc;
		nc.valid.reserve(keep.size());
		for (int64_t s : keep) nc.valid.push_back(c.valid[(size_t)s]);
		if (c.type == COL_INT || c.type == COL_BOOL)
			for (int64_t s : keep) nc.i.push_back(c.i[(size_t)s]);
		if (c.type == COL_FLOAT)
			for (int64_t s : keep) nc.f.push_back(c.f[(size_t)s]);
		if (c.type == COL_STRING)
			for (int64_t s : keep) nc.s.push_back(std::move(c.s[(size_t)s]));
		c.valid.swap(nc.valid);
		c.i.swap(nc.i);
		c.f.swap(nc.f);
		c.s.swap(nc.s);
		if (c.index) c.build_index(c.index->type);  // slots moved
	}
}

// total order of the index: NaN after every number (DataFusion's order), ties by slot
void MetaColumn::build_index(const std::string &ty) {
	auto ix = std::make_shared<ColIndex>();
	ix->type = ty;
	ix->n_indexed = (int64_t)size();
	for (int64_t r = 0; r < ix->n_indexed; ++r)
		if (valid[(size_t)r]) ix->perm.push_back((uint32_t)r);
	auto less = [&](uint32_t a, uint32_t b) {
		switch (type) {
		case COL_INT:
		case COL_BOOL:
			if (i[a] != i[b]) return i[a] < i[b];
			break;
		case COL_FLOAT: {
			const double x = f[a], y = f[b];
			const bool nx = std::isnan(x), ny = std::isnan(y);
			if (nx != ny) return ny;
			if (!nx && x != y) return x < y;
			break;
		}
		case COL_STRING: {
			const int c = s[a].compare(s[b]);
			if (c != 0) return c < 0;
			break;
		}
		}
		return a < b;
	};
	std::sort(ix->perm.begin(), ix->perm.end(), less);
	index = ix;
}

void MetaStore::append_rows(const MetaStore &src, const std::vector<int64_t> &src_slots) {
	if (src.cols.size() != cols.size()) throw Error("merged indexes have different metadata columns");
	for (size_t c = 0; c < cols.size(); ++c) {
		MetaColumn &d = cols[c];
		const MetaColumn &s = src.cols[c];
		if (d.type != s.type || d.name != s.name) throw Error("merged indexes have different metadata columns");
		for (int64_t r : src_slots) {
			d.valid.push_back(s.valid[(size_t)r]);
			if (d.type == COL_INT || d.type == COL_BOOL) d.i.push_back(s.i[(size_t)r]);
			if (d.type == COL_FLOAT) d.f.push_back(s.f[(size_t)r]);
			if (d.type == COL_STRING) d.s.push_back(s.s[(size_t)r]);
		}
	}
}

void MetaStore::truncate(size_t n) {
	for (auto &c : cols) {
		c.valid.resize(std::min(n, c.valid.size()));
		if (c.type == COL_INT || c.type == COL_BOOL) c.i.resize(c.valid.size());
		if (c.type == COL_FLOAT) c.f.resize(c.valid.size());
		if (c.type == COL_STRING) c.s.resize(c.valid.size());
	}
}

void MetaStore::append_nulls(int64_t n) {
	for (auto &c : cols) {
		c.valid.insert(c.valid.end(), (size_t)n, 0);
		if (c.type == COL_INT || c.type == COL_BOOL) c.i.insert(c.i.end(), (size_t)n, 0);
		if (c.type == COL_FLOAT) c.f.insert(c.f.end(), (size_t)n, 0.0);
		if (c.type == COL_STRING) c.s.insert(c.s.end(), (size_t)n, std::string());
	}
}

// ---- persistence (a record per ingest batch in the table log) --------------
static void put(std::vector<uint8_t> &o, const void *p, size_t n) {
	const uint8_t *b = static_cast<const uint8_t *>(p);
	o.insert(o.end(), b, b + n);
}
template <typename T>
static void put_v(std::vector<uint8_t> &o, T v) {
	put(o, &v, sizeof(T));
}
struct Reader {
	const uint8_t *p, *e;
	void get(void *d, size_t n) {
		if ((size_t)(e - p) < n) throw Error("corrupt metadata record");
		memcpy(d, p, n);
		p += n;
	}
	template <typename T>
	T v() {
		T x;
		get(&x, sizeof(T));
		return x;
	}
	std::string str() {
		const uint32_t n = v<uint32_t>();
		if ((size_t)(e - p) < n) throw Error("corrupt metadata record");
		std::string s(reinterpret_cast<const char *>(p), n);
		p += n;
		return s;
	}
};
static void put_s(std::vector<uint8_t> &o, const std::string &s) {
	put_v<uint32_t>(o, (uint32_t)s.size());
	put(o, s.data(), s.size());
}

void MetaStore::serialize_schema(std::vector<uint8_t> &out) const {
	put_s(out, vector_name);
	put_v<int32_t>(out, vector_pos);
	put_v<int32_t>(out, dim);
	put_v<int32_t>(out, (int32_t)cols.size());
	for (auto &c : cols) {
		put_s(out, c.name);
		put_s(out, c.arrow_format);
		put_v<int32_t>(out, (int32_t)c.type);
	}
}

std::unique_ptr<MetaStore> MetaStore::deserialize_schema(const uint8_t *p, size_t len) {
	Reader r{p, p + len};
	auto m = std::make_unique<MetaStore>();
	m->vector_name = r.str();
	m->vector_pos = r.v<int32_t>();
	m->dim = r.v<int32_t>();
	const int nc = r.v<int32_t>();
	for (int i = 0; i < nc; ++i) {
		MetaColumn c;
		c.name = r.str();
		c.arrow_format = r.str();
		c.type = (ColType)r.v<int32_t>();
		m->cols.push_back(std::move(c));
	}
	return m;
}

void MetaStore::serialize_rows(int64_t s0, int64_t n, std::vector<uint8_t> &out) const {
	put_v<int64_t>(out, n);
	for (auto &c : cols) {
		put(out, c.valid.data() + s0, (size_t)n);
		if (c.type == COL_INT || c.type == COL_BOOL) put(out, c.i.data() + s0, (size_t)n * 8);
		if (c.type == COL_FLOAT) put(out, c.f.data() + s0, (size_t)n * 8);
		if (c.type == COL_STRING)
			for (int64_t r = 0; r < n; ++r) put_s(out, c.s[(size_t)(s0 + r)]);
	}
}

void MetaStore::deserialize_rows(const uint8_t *p, size_t len) {
	Reader r{p, p + len};
	const int64_t n = r.v<int64_t>();
	for (auto &c : cols) {
		const size_t b = c.valid.size();
		c.valid.resize(b + (size_t)n);
		r.get(c.valid.data() + b, (size_t)n);
		if (c.type == COL_INT || c.type == COL_BOOL) {
			c.i.resize(b + (size_t)n);
			r.get(c.i.data() + b, (size_t)n * 8);
		}
		if (c.type == COL_FLOAT) {
			c.f.resize(b + (size_t)n);
			r.get(c.f.data() + b, (size_t)n * 8);
		}
		if (c.type == COL_STRING)
			for (int64_t k = 0; k < n; ++k) c.s.push_back(r.str());
	}
}

// ---------------------------------------------------------------------------
// predicate: tokenizer, parser, vectorised three-valued evaluation
// ---------------------------------------------------------------------------
namespace {

enum Tri : uint8_t { T_FALSE = 0, T_TRUE = 1, T_NULL = 2 };

struct Tok {
	enum Kind { IDENT, STR, NUM, OP, LP, RP, COMMA, END } kind;
	std::string text;  // IDENT: as written (keywords matched case-insensitively)
};

static std::string upper(std::string s) {
	for (auto &ch : s) ch = (char)toupper((unsigned char)ch);
	return s;
}

static std::vector<Tok> tokenize(const std::string &src) {
	std::vector<Tok> out;
	size_t i = 0;
	while (i < src.size()) {
		const char c = src[i];
		if (isspace((unsigned char)c)) {
			++i;
		} else if (c == '(') {
			out.push_back({Tok::LP, "("});
			++i;
		} else if (c == ')') {
			out.push_back({Tok::RP, ")"});
			++i;
		} else if (c == ',') {
			out.push_back({Tok::COMMA, ","});
			++i;
		} else if (c == '\'') {  // 'it''s'
			std::string s;
			++i;
			for (;;) {
				if (i >= src.size()) throw Error("predicate: unterminated string literal");
				if (src[i] == '\'') {
					if (i + 1 < src.size() && src[i + 1] == '\'') {
						s += '\'';
						i += 2;
						continue;
					}
					++i;
					break;
				}
				s += src[i++];
			}
			out.push_back({Tok::STR, s});
		} else if (c == '"' || c == '`') {  // quoted identifier
			const char q = c;
			std::string s;
			++i;
			while (i < src.size() && src[i] != q) s += src[i++];
			if (i >= src.size()) throw Error("predicate: unterminated quoted identifier");
			++i;
			out.push_back({Tok::IDENT, s});
		} else if (isdigit((unsigned char)c) || (c == '.' && i + 1 < src.size() && isdigit((unsigned char)src[i + 1])) ||
		           (c == '-' && i + 1 < src.size() &&
		            (isdigit((unsigned char)src[i + 1]) || src[i + 1] == '.') &&
		            (out.empty() || out.back().kind == Tok::OP || out.back().kind == Tok::LP ||
		             out.back().kind == Tok::COMMA ||
		             (out.back().kind == Tok::IDENT && (upper(out.back().text) == "AND" ||
		                                                upper(out.back().text) == "OR" ||
		                                                upper(out.back().text) == "NOT" ||
		                                                upper(out.back().text) == "BETWEEN" ||
		                                                upper(out.back().text) == "IN"))))) {
			size_t j = i + 1;
			while (j < src.size() && (isalnum((unsigned char)src[j]) || src[j] == '.' ||
			                          ((src[j] == '+' || src[j] == '-') && (src[j - 1] == 'e' || src[j - 1] == 'E'))))
				++j;
			out.push_back({Tok::NUM, src.substr(i, j - i)});
			i = j;
		} else if (isalpha((unsigned char)c) || c == '_') {
			size_t j = i + 1;
			while (j < src.size() && (isalnum((unsigned char)src[j]) || src[j] == '_')) ++j;
			out.push_back({Tok::IDENT, src.substr(i, j - i)});
			i = j;
		} else {
			static const char *ops[] = {"<=", ">=", "!=", "<>", "==", "=", "<", ">"};
			bool hit = false;
			for (const char *op : ops) {
				const size_t n = strlen(op);
				if (src.compare(i, n, op) == 0) {
					out.push_back({Tok::OP, op});
					i += n;
					hit = true;
					break;
				}
			}
			if (!hit) throw Error(std::string("predicate: unexpected character '") + c + "'");
		}
	}
	out.push_back({Tok::END, ""});
	return out;
}

struct Value {
	enum Kind { NUL, INT, FLT, BOOL, STR } kind = NUL;
	int64_t i = 0;
	double f = 0.0;
	std::string s;
};

struct Node;
using NodeP = std::unique_ptr<Node>;
struct Node {
	enum Kind { AND, OR, NOT, CMP, ISNULL, IN, COL, LIT } kind;
	std::string op;     // CMP
	bool neg = false;   // ISNULL (IS NOT NULL), IN (NOT IN)
	std::vector<NodeP> kids;
	std::string col;    // COL
	Value lit;          // LIT
};

struct Parser {
	std::vector<Tok> t;
	size_t p = 0;
	const Tok &peek() const { return t[p]; }
	bool kw(const char *k) const { return t[p].kind == Tok::IDENT && upper(t[p].text) == k; }
	bool kw_at(size_t q, const char *k) const { return q < t.size() && t[q].kind == Tok::IDENT && upper(t[q].text) == k; }
	void expect(Tok::Kind k, const char *what) {
		if (t[p].kind != k) throw Error(std::string("predicate: expected ") + what + " near '" + t[p].text + "'");
		++p;
	}
	NodeP mk(Node::Kind k) {
		auto n = std::make_unique<Node>();
		n->kind = k;
		return n;
	}
	NodeP expr() { return or_(); }
	NodeP or_() {
		NodeP a = and_();
		while (kw("OR")) {
			++p;
			NodeP n = mk(Node::OR);
			n->kids.push_back(std::move(a));
			n->kids.push_back(and_());
			a = std::move(n);
		}
		return a;
	}
	NodeP and_() {
		NodeP a = not_();
		while (kw("AND")) {
			++p;
			NodeP n = mk(Node::AND);
			n->kids.push_back(std::move(a));
			n->kids.push_back(not_());
			a = std::move(n);
		}
		return a;
	}
	NodeP not_() {
		if (kw("NOT")) {
			++p;
			NodeP n = mk(Node::NOT);
			n->kids.push_back(not_());
			return n;
		}
		return pred();
	}
	NodeP operand() {
		const Tok &k = peek();
		if (k.kind == Tok::LP) {
			++p;
			NodeP e = expr();
			expect(Tok::RP, "')'");
			return e;
		}
		NodeP n = mk(Node::LIT);
		if (k.kind == Tok::STR) {
			n->lit.kind = Value::STR;
			n->lit.s = k.text;
		} else if (k.kind == Tok::NUM) {
			const std::string &x = k.text;
			if (x.find_first_of(".eE") == std::string::npos) {
				n->lit.kind = Value::INT;
				n->lit.i = strtoll(x.c_str(), nullptr, 10);
			} else {
				n->lit.kind = Value::FLT;
				n->lit.f = strtod(x.c_str(), nullptr);
			}
		} else if (k.kind == Tok::IDENT) {
			const std::string u = upper(k.text);
			if (u == "NULL") {
				n->lit.kind = Value::NUL;
			} else if (u == "TRUE" || u == "FALSE") {
				n->lit.kind = Value::BOOL;
				n->lit.i = u == "TRUE";
			} else if (u == "AND" || u == "OR" || u == "NOT" || u == "IS" || u == "IN" || u == "BETWEEN") {
				throw Error("predicate: unexpected keyword '" + k.text + "'");
			} else {
				n->kind = Node::COL;
				n->col = k.text;
			}
		} else {
			throw Error("predicate: expected a column or a literal near '" + k.text + "'");
		}
		++p;
		return n;
	}
	NodeP pred() {
		NodeP a = operand();
		if (peek().kind == Tok::OP) {
			std::string op = peek().text;
			++p;
			if (op == "<>") op = "!=";
			if (op == "==") op = "=";
			NodeP n = mk(Node::CMP);
			n->op = op;
			n->kids.push_back(std::move(a));
			n->kids.push_back(operand());
			return n;
		}
		if (kw("IS")) {
			++p;
			NodeP n = mk(Node::ISNULL);
			if (kw("NOT")) {
				++p;
				n->neg = true;
			}
			if (!kw("NULL")) throw Error("predicate: expected NULL after IS");
			++p;
			n->kids.push_back(std::move(a));
			return n;
		}
		bool neg = false;
		if (kw("NOT") && (kw_at(p + 1, "IN") || kw_at(p + 1, "BETWEEN"))) {
			neg = true;
			++p;
		}
		if (kw("IN")) {
			++p;
			NodeP n = mk(Node::IN);
			n->neg = neg;
			n->kids.push_back(std::move(a));
			expect(Tok::LP, "'('");
			for (;;) {
				n->kids.push_back(operand());
				if (peek().kind == Tok::COMMA) {
					++p;
					continue;
				}
				break;
			}
			expect(Tok::RP, "')'");
			return n;
		}
		if (kw("BETWEEN")) {  // a BETWEEN lo AND hi  ==  a >= lo AND a <= hi
			++p;
			NodeP lo = operand();
			if (!kw("AND")) throw Error("predicate: expected AND in BETWEEN");
			++p;
			NodeP hi = operand();
			auto cmp = [&](const char *op, NodeP x, NodeP y) {
				NodeP c = mk(Node::CMP);
				c->op = op;
				c->kids.push_back(std::move(x));
				c->kids.push_back(std::move(y));
				return c;
			};
			auto copy_operand = [&](const Node &src) {
				NodeP c = mk(src.kind);
				c->col = src.col;
				c->lit = src.lit;
				if (src.kind != Node::COL && src.kind != Node::LIT)
					throw Error("predicate: BETWEEN needs a column or literal operand");
				return c;
			};
			NodeP a2 = copy_operand(*a);
			NodeP n = mk(Node::AND);
			n->kids.push_back(cmp(">=", std::move(a), std::move(lo)));
			n->kids.push_back(cmp("<=", std::move(a2), std::move(hi)));
			if (!neg) return n;
			NodeP nn = mk(Node::NOT);
			nn->kids.push_back(std::move(n));
			return nn;
		}
		if (neg) throw Error("predicate: expected IN or BETWEEN after NOT");
		return a;  // a bare column or literal used as a boolean
	}
};

// vectorised evaluation over n slots
struct Eval {
	const MetaStore *meta;
	const std::vector<int64_t> &labels;
	size_t n;

	struct ColRef {
		ColType type;
		const std::vector<int64_t> *i = nullptr;
		const std::vector<double> *f = nullptr;
		const std::vector<std::string> *s = nullptr;
		const std::vector<uint8_t> *valid = nullptr;  // null = all valid
		const ColIndex *index = nullptr;
	};
	ColRef column(const std::string &name) const {
		if (meta)
			for (auto &c : meta->cols)
				if (c.name == name) return ColRef{c.type, &c.i, &c.f, &c.s, &c.valid, c.index.get()};
		if (name == "label") return ColRef{COL_INT, &labels, nullptr, nullptr, nullptr};
		if (meta)
			for (auto &c : meta->cols)  // DataFusion folds unquoted identifiers to lower case
				if (upper(c.name) == upper(name)) return ColRef{c.type, &c.i, &c.f, &c.s, &c.valid, c.index.get()};
		throw Error("predicate: no column named '" + name + "'");
	}
	static Value at(const ColRef &c, size_t r) {
		Value v;
		if (c.valid && !(*c.valid)[r]) return v;
		switch (c.type) {
		case COL_INT: v.kind = Value::INT; v.i = (*c.i)[r]; break;
		case COL_BOOL: v.kind = Value::BOOL; v.i = (*c.i)[r]; break;
		case COL_FLOAT: v.kind = Value::FLT; v.f = (*c.f)[r]; break;
		case COL_STRING: v.kind = Value::STR; v.s = (*c.s)[r]; break;
		}
		return v;
	}
	// three-valued compare of two non-null values
	static bool cmp_vals(const Value &a, const Value &b, const std::string &op) {
		int c;
		if (a.kind == Value::STR || b.kind == Value::STR) {
			if (a.kind != b.kind) throw Error("predicate: cannot compare a string with a non-string");
			c = a.s.compare(b.s);
			c = c < 0 ? -1 : c > 0;
		} else if (a.kind == Value::BOOL || b.kind == Value::BOOL) {
			if (a.kind != b.kind) throw Error("predicate: cannot compare a boolean with a non-boolean");
			c = (a.i > b.i) - (a.i < b.i);
		} else if (a.kind == Value::INT && b.kind == Value::INT) {
			c = (a.i > b.i) - (a.i < b.i);
		} else {
			const double x = a.kind == Value::INT ? (double)a.i : a.f, y = b.kind == Value::INT ? (double)b.i : b.f;
			if (std::isnan(x) || std::isnan(y)) {  // DataFusion total order: NaN is the largest
				c = std::isnan(x) && std::isnan(y) ? 0 : (std::isnan(x) ? 1 : -1);
			} else {
				c = (x > y) - (x < y);
			}
		}
		if (op == "=") return c == 0;
		if (op == "!=") return c != 0;
		if (op == "<") return c < 0;
		if (op == "<=") return c <= 0;
		if (op == ">") return c > 0;
		return c >= 0;
	}
	static const char *flip(const std::string &op) {
		if (op == "<") return ">";
		if (op == "<=") return ">=";
		if (op == ">") return "<";
		if (op == ">=") return "<=";
		return op == "=" ? "=" : "!=";
	}

	std::vector<uint8_t> cmp(const Node &x) {
		const Node &a = *x.kids[0], &b = *x.kids[1];
		std::vector<uint8_t> out(n, T_NULL);
		if (a.kind == Node::LIT && b.kind == Node::LIT) {
			if (a.lit.kind != Value::NUL && b.lit.kind != Value::NUL)
				std::fill(out.begin(), out.end(), cmp_vals(a.lit, b.lit, x.op) ? T_TRUE : T_FALSE);
			return out;
		}
		if (a.kind == Node::COL && b.kind == Node::LIT) return cmp_col_lit(column(a.col), b.lit, x.op);
		if (a.kind == Node::LIT && b.kind == Node::COL) return cmp_col_lit(column(b.col), a.lit, flip(x.op));
		if (a.kind == Node::COL && b.kind == Node::COL) {
			const ColRef ca = column(a.col), cb = column(b.col);
			for (size_t r = 0; r < n; ++r) {
				const Value va = at(ca, r), vb = at(cb, r);
				if (va.kind != Value::NUL && vb.kind != Value::NUL) out[r] = cmp_vals(va, vb, x.op) ? T_TRUE : T_FALSE;
			}
			return out;
		}
		throw Error("predicate: comparison operands must be columns or literals");
	}
	// indexed column vs literal: the rows of [0, n_indexed) that satisfy the
	// comparison are one or two ranges of the sorted permutation
	bool cmp_indexed(const ColRef &c, const Value &lit, const std::string &op, std::vector<uint8_t> &out) {
		const ColIndex &ix = *c.index;
		const bool str = c.type == COL_STRING, lstr = lit.kind == Value::STR;
		if (str != lstr) return false;                                  // type error: generic path reports it
		if ((c.type == COL_BOOL) != (lit.kind == Value::BOOL)) return false;
		if (c.type == COL_INT && lit.kind == Value::FLT) return false;  // mixed int / float: generic path
		// sign of (value of perm[p]) - literal, monotone in p
		auto sgn = [&](uint32_t r) -> int {
			if (str) {
				const int k = (*c.s)[r].compare(lit.s);
				return k < 0 ? -1 : k > 0;
			}
			if (c.type == COL_FLOAT) {
				const double x = (*c.f)[r], y = lit.kind == Value::INT ? (double)lit.i : lit.f;
				if (std::isnan(x) || std::isnan(y)) return std::isnan(x) && std::isnan(y) ? 0 : (std::isnan(x) ? 1 : -1);
				return (x > y) - (x < y);
			}
			const int64_t x = (*c.i)[r], y = lit.i;
			return (x > y) - (x < y);
		};
		const auto &pm = ix.perm;
		const size_t lo = std::partition_point(pm.begin(), pm.end(), [&](uint32_t r) { return sgn(r) < 0; }) - pm.begin();
		const size_t hi = std::partition_point(pm.begin() + lo, pm.end(), [&](uint32_t r) { return sgn(r) == 0; }) - pm.begin();
		// [0, lo) < lit, [lo, hi) == lit, [hi, end) > lit
		const size_t ni = (size_t)std::min<int64_t>(ix.n_indexed, (int64_t)n);
		for (size_t r = 0; r < ni; ++r) out[r] = (!c.valid || (*c.valid)[r]) ? T_FALSE : T_NULL;
		auto mark = [&](size_t a, size_t b) {
			for (size_t p = a; p < b; ++p)
				if (pm[p] < ni) out[pm[p]] = T_TRUE;
		};
		if (op == "=") mark(lo, hi);
		else if (op == "!=") { mark(0, lo); mark(hi, pm.size()); }
		else if (op == "<") mark(0, lo);
		else if (op == "<=") mark(0, hi);
		else if (op == ">") mark(hi, pm.size());
		else mark(lo, pm.size());
		for (size_t r = ni; r < n; ++r) {  // rows appended after the index was built
			if (c.valid && !(*c.valid)[r]) continue;
			out[r] = cmp_vals(at(c, r), lit, op) ? T_TRUE : T_FALSE;
		}
		return true;
	}
	std::vector<uint8_t> cmp_col_lit(const ColRef &c, const Value &lit, const std::string &op) {
		std::vector<uint8_t> out(n, T_NULL);
		if (lit.kind == Value::NUL) return out;
		if (c.index && cmp_indexed(c, lit, op, out)) return out;
		auto valid = [&](size_t r) { return !c.valid || (*c.valid)[r]; };
		if (c.type == COL_INT && lit.kind == Value::INT) {  // exact int64 compare
			const int64_t y = lit.i;
			for (size_t r = 0; r < n; ++r) {
				if (!valid(r)) continue;
				const int64_t v = (*c.i)[r];
				const int k = (v > y) - (v < y);
				bool t;
				if (op == "=") t = k == 0;
				else if (op == "!=") t = k != 0;
				else if (op == "<") t = k < 0;
				else if (op == "<=") t = k <= 0;
				else if (op == ">") t = k > 0;
				else t = k >= 0;
				out[r] = t ? T_TRUE : T_FALSE;
			}
			return out;
		}
		for (size_t r = 0; r < n; ++r) {
			if (!valid(r)) continue;
			out[r] = cmp_vals(at(c, r), lit, op) ? T_TRUE : T_FALSE;
		}
		return out;
	}
	std::vector<uint8_t> run(const Node &x) {
		switch (x.kind) {
		case Node::AND:
		case Node::OR: {
			std::vector<uint8_t> a = run(*x.kids[0]), b = run(*x.kids[1]);
			for (size_t r = 0; r < n; ++r) {
				if (x.kind == Node::AND)
					a[r] = (a[r] == T_FALSE || b[r] == T_FALSE) ? T_FALSE : (a[r] == T_TRUE && b[r] == T_TRUE) ? T_TRUE : T_NULL;
				else
					a[r] = (a[r] == T_TRUE || b[r] == T_TRUE) ? T_TRUE : (a[r] == T_FALSE && b[r] == T_FALSE) ? T_FALSE : T_NULL;
			}
			return a;
		}
		case Node::NOT: {
			std::vector<uint8_t> a = run(*x.kids[0]);
			for (auto &v : a) v = v == T_NULL ? T_NULL : (uint8_t)(1 - v);
			return a;
		}
		case Node::CMP: return cmp(x);
		case Node::ISNULL: {
			const Node &a = *x.kids[0];
			std::vector<uint8_t> out(n);
			if (a.kind == Node::LIT) {
				std::fill(out.begin(), out.end(), ((a.lit.kind == Value::NUL) != x.neg) ? T_TRUE : T_FALSE);
			} else if (a.kind == Node::COL) {
				const ColRef c = column(a.col);
				for (size_t r = 0; r < n; ++r) {
					const bool isnull = c.valid && !(*c.valid)[r];
					out[r] = (isnull != x.neg) ? T_TRUE : T_FALSE;
				}
			} else {
				std::vector<uint8_t> v = run(a);
				for (size_t r = 0; r < n; ++r) out[r] = ((v[r] == T_NULL) != x.neg) ? T_TRUE : T_FALSE;
			}
			return out;
		}
		case Node::IN: {  // a IN (l1, l2, ..) == a = l1 OR a = l2 ...; NOT IN = NOT (that)
			std::vector<uint8_t> acc(n, T_FALSE);
			for (size_t i = 1; i < x.kids.size(); ++i) {
				Node eq;
				eq.kind = Node::CMP;
				eq.op = "=";
				auto l = std::make_unique<Node>();
				l->kind = x.kids[0]->kind;
				l->col = x.kids[0]->col;
				l->lit = x.kids[0]->lit;
				auto r = std::make_unique<Node>();
				r->kind = x.kids[i]->kind;
				r->col = x.kids[i]->col;
				r->lit = x.kids[i]->lit;
				eq.kids.push_back(std::move(l));
				eq.kids.push_back(std::move(r));
				const std::vector<uint8_t> b = cmp(eq);
				for (size_t k = 0; k < n; ++k)
					acc[k] = (acc[k] == T_TRUE || b[k] == T_TRUE) ? T_TRUE
					         : (acc[k] == T_FALSE && b[k] == T_FALSE) ? T_FALSE : T_NULL;
			}
			if (x.neg)
				for (auto &v : acc) v = v == T_NULL ? T_NULL : (uint8_t)(1 - v);
			return acc;
		}
		case Node::COL: {  // a boolean column used as a predicate
			const ColRef c = column(x.col);
			if (c.type != COL_BOOL) throw Error("predicate: column '" + x.col + "' is not boolean");
			std::vector<uint8_t> out(n, T_NULL);
			for (size_t r = 0; r < n; ++r)
				if (!c.valid || (*c.valid)[r]) out[r] = (*c.i)[r] ? T_TRUE : T_FALSE;
			return out;
		}
		case Node::LIT: {
			if (x.lit.kind != Value::BOOL && x.lit.kind != Value::NUL) throw Error("predicate: not a boolean expression");
			return std::vector<uint8_t>(n, x.lit.kind == Value::NUL ? T_NULL : (x.lit.i ? T_TRUE : T_FALSE));
		}
		}
		return std::vector<uint8_t>(n, T_NULL);
	}
};

}  // namespace

int64_t eval_predicate(const std::string &predicate, const MetaStore *meta, const std::vector<int64_t> &labels,
                       const std::vector<uint8_t> &live, std::vector<uint8_t> &mask) {
	Parser ps{tokenize(predicate)};
	NodeP root = ps.expr();
	if (ps.peek().kind != Tok::END) throw Error("predicate: unexpected '" + ps.peek().text + "'");
	Eval ev{meta, labels, labels.size()};
	std::vector<uint8_t> tri = ev.run(*root);
	mask.assign(labels.size(), 0);
	int64_t cnt = 0;
	for (size_t s = 0; s < labels.size(); ++s)
		if (live[s] && tri[s] == T_TRUE) {
			mask[s] = 1;
			++cnt;
		}
	return cnt;
}

}  // namespace lhip
