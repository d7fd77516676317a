// dlp_general.cpp — general LPs for the GPU simplex:
// the canonical standard form (row / column bounds -> L/G/E rows over x' >= 0,
// slack / surplus / artificial columns) and a free/fixed MPS reader.  Host-side
// problem formulation only; every pivot of both phases runs in the HIP kernels
// (dlp_kernels.hip) driven by dlp_session.cpp.
//
// The reference has no file input and no general LP: it builds its own
// ad-allocation instance in memory (R/instance.cpp:32-57) and prints errors
// and carries on.  This module returns DLP_ERR_* codes with
// a dlp_last_error() message instead, as the rest of the C ABI does.
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "dlp_host.h"

namespace dlp {
namespace {

inline bool infinite(double v) { return !(std::fabs(v) < 1e30); }

// Negation of a standard row: v -> 0.0 - v, so zeros stay +0.0.
inline double neg(double v) { return 0.0 - v; }

struct Row {
    std::vector<double> a;   // ns coefficients
    double rhs;
    int8_t type;
    int32_t user;
};

}  // namespace

int build_stdform(const General& g, StdForm* out) {
    StdForm& s = *out;
    s = StdForm();
    const int64_t m = g.m, n = g.n;
    // ---- columns
    s.var_col.resize(n);
    s.var_kind.resize(n);
    s.var_const.assign(n, 0.0);
    for (int64_t j = 0; j < n; ++j) {
        const double lo = g.col_lo[j], hi = g.col_hi[j];
        if (std::isnan(lo) || std::isnan(hi) || (infinite(lo) && lo > 0) || (infinite(hi) && hi < 0)) {
            set_error("column " + std::to_string(j) + ": invalid bounds");
            return DLP_ERR_ARG;
        }
        s.var_col[j] = (int32_t)s.ns;
        if (!infinite(lo)) {
            s.var_kind[j] = VAR_LO;
            s.var_const[j] = lo;
            s.ns += 1;
        } else if (!infinite(hi)) {
            s.var_kind[j] = VAR_HI;
            s.var_const[j] = hi;
            s.ns += 1;
        } else {
            s.var_kind[j] = VAR_FREE;
            s.ns += 2;
        }
    }
    const int64_t ns = s.ns;
    if (ns + 1 > INT32_MAX) { set_error("too many columns"); return DLP_ERR_ARG; }
    s.c.assign(ns, 0.0);
    for (int64_t j = 0; j < n; ++j) {
        const double base = g.sense == DLP_MINIMIZE ? -g.c[j] : g.c[j];
        const int32_t k = s.var_col[j];
        if (s.var_kind[j] == VAR_LO) {
            s.c[k] = base;
        } else if (s.var_kind[j] == VAR_HI) {
            s.c[k] = -base;
        } else {
            s.c[k] = base;
            s.c[k + 1] = -base;
        }
    }

    s.obj_sign = g.sense == DLP_MINIMIZE ? -1.0 : 1.0;
    double cshift = 0.0;
    for (int64_t j = 0; j < n; ++j)
        if (s.var_kind[j] != VAR_FREE) cshift = std::fma(g.c[j], s.var_const[j], cshift);
    s.obj_const = g.c0 + cshift;

    // ---- rows: user rows in order, then bound rows in column order
    std::vector<Row> rows;
    for (int64_t i = 0; i < m; ++i) {
        const double rl = g.row_lo[i], ru = g.row_hi[i];
        if (std::isnan(rl) || std::isnan(ru) || (infinite(rl) && rl > 0) || (infinite(ru) && ru < 0)) {
            set_error("row " + std::to_string(i) + ": invalid bounds");
            return DLP_ERR_ARG;
        }
        if (infinite(rl) && infinite(ru)) continue;   // free row: no constraint
        Row r;
        r.a.assign(ns, 0.0);
        r.user = (int32_t)i;
        double shift = 0.0;
        const double* Ai = g.A.data() + i * n;
        for (int64_t j = 0; j < n; ++j) {
            const double a = Ai[j];
            if (std::isnan(a)) { set_error("A has a NaN"); return DLP_ERR_ARG; }
            const int32_t k = s.var_col[j];
            switch (s.var_kind[j]) {
                case VAR_LO: r.a[k] = a; shift = std::fma(a, s.var_const[j], shift); break;
                case VAR_HI: r.a[k] = -a; shift = std::fma(a, s.var_const[j], shift); break;
                default: r.a[k] = a; r.a[k + 1] = -a; break;
            }
        }
        if (!infinite(rl) && !infinite(ru) && rl == ru) {
            r.type = ROW_E;
            r.rhs = rl - shift;
            rows.push_back(r);
        } else {
            if (!infinite(ru)) {
                r.type = ROW_L;
                r.rhs = ru - shift;
                rows.push_back(r);
            }
            if (!infinite(rl)) {
                r.type = ROW_G;
                r.rhs = rl - shift;
                rows.push_back(r);
            }
        }
    }
    for (int64_t j = 0; j < n; ++j) {
        if (s.var_kind[j] != VAR_LO || infinite(g.col_hi[j])) continue;
        Row r;
        r.a.assign(ns, 0.0);
        r.a[s.var_col[j]] = 1.0;
        r.rhs = g.col_hi[j] - g.col_lo[j];
        r.type = ROW_L;
        r.user = -1;
        rows.push_back(r);
    }
    if (rows.empty()) {
        set_error("the LP has no constraint rows after canonicalisation (only free / lower-bounded "
                  "variables and free rows)");
        return DLP_ERR_UNSUPPORTED;
    }

    // ---- normalise signs, assign slack / surplus / artificial columns
    s.m = (int64_t)rows.size();
    s.A.assign((size_t)s.m * ns, 0.0);
    s.b.resize(s.m);
    s.type.resize(s.m);
    s.user_row.resize(s.m);
    s.row_sign.resize(s.m);
    s.slack_col.assign(s.m, -1);
    s.art_col.assign(s.m, -1);
    for (int64_t i = 0; i < s.m; ++i) {
        Row& r = rows[i];
        double sign = 1.0;
        const bool flip = r.rhs < 0.0 || (r.rhs == 0.0 && r.type == ROW_G);
        if (flip) {
            for (double& v : r.a) v = neg(v);
            r.rhs = neg(r.rhs);
            if (r.type == ROW_L) r.type = ROW_G;
            else if (r.type == ROW_G) r.type = ROW_L;
            sign = -1.0;
        }
        r.rhs = r.rhs + 0.0;   // -0.0 -> +0.0
        std::memcpy(s.A.data() + i * ns, r.a.data(), sizeof(double) * ns);
        s.b[i] = r.rhs;
        s.type[i] = r.type;
        s.user_row[i] = r.user;
        s.row_sign[i] = sign;
        if (r.type != ROW_E) s.nslack += 1;
        if (r.type != ROW_L) s.nart += 1;
    }
    int64_t ks = ns, ka = ns + s.nslack;
    for (int64_t i = 0; i < s.m; ++i) {
        if (s.type[i] != ROW_E) s.slack_col[i] = (int32_t)ks++;
        if (s.type[i] != ROW_L) s.art_col[i] = (int32_t)ka++;
    }
    if (s.ncols() + 1 > INT32_MAX) { set_error("too many columns"); return DLP_ERR_ARG; }
    return DLP_OK;
}

// ------------------------------------------------------------------ MPS
namespace {

std::vector<std::string> split(const char* line) {
    std::vector<std::string> t;
    const char* p = line;
    while (*p) {
        while (*p && std::isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        const char* q = p;
        while (*q && !std::isspace((unsigned char)*q)) ++q;
        t.emplace_back(p, q - p);
        p = q;
    }
    return t;
}

std::string upper(std::string s) {
    for (char& ch : s) ch = (char)std::toupper((unsigned char)ch);
    return s;
}

bool number(const std::string& s, double* v) {
    char* end = nullptr;
    *v = std::strtod(s.c_str(), &end);
    return end && *end == '\0' && end != s.c_str();
}

}  // namespace

int parse_mps(const char* path, General* out) {
    FILE* f = std::fopen(path, "r");
    if (!f) {
        set_error(std::string("cannot open MPS file ") + path);
        return DLP_ERR_ARG;
    }
    enum Sec { NONE, NAME, OBJSENSE, ROWS, COLUMNS, RHS, RANGES, BOUNDS, END } sec = NONE;
    std::unordered_map<std::string, int64_t> row_id, col_id;   // row id: >= 0, -1 objective, -2 dropped N row
    std::vector<char> rtype;
    std::vector<double> rhs, range;
    std::vector<bool> has_range;
    std::vector<double> c, lo, hi;
    struct Entry { int64_t i, j; double v; };
    std::vector<Entry> entries;
    std::string objname;
    int sense = DLP_MINIMIZE;
    double c0 = 0.0;
    int64_t lineno = 0;
    std::string err;
    char buf[65536];

    auto fail = [&](const std::string& msg) {
        err = "MPS line " + std::to_string(lineno) + ": " + msg;
    };
    auto row_of = [&](const std::string& name, int64_t* id) -> bool {
        auto it = row_id.find(name);
        if (it == row_id.end()) { fail("unknown row " + name); return false; }
        *id = it->second;
        return true;
    };
    auto col_of = [&](const std::string& name, int64_t* id) -> bool {
        auto it = col_id.find(name);
        if (it == col_id.end()) { fail("unknown column " + name); return false; }
        *id = it->second;
        return true;
    };

    while (err.empty() && sec != END && std::fgets(buf, sizeof(buf), f)) {
        ++lineno;
        const size_t len = std::strlen(buf);
        if (len == sizeof(buf) - 1 && buf[len - 1] != '\n') { fail("line too long"); break; }
        if (buf[0] == '*' || buf[0] == '\n' || buf[0] == '\r' || buf[0] == '\0') continue;
        auto t = split(buf);
        if (t.empty()) continue;
        if (!std::isspace((unsigned char)buf[0])) {   // section header
            const std::string h = upper(t[0]);
            if (h == "NAME") sec = NAME;
            else if (h == "ROWS") sec = ROWS;
            else if (h == "COLUMNS") sec = COLUMNS;
            else if (h == "RHS") sec = RHS;
            else if (h == "RANGES") sec = RANGES;
            else if (h == "BOUNDS") sec = BOUNDS;
            else if (h == "ENDATA") sec = END;
            else if (h == "OBJSENSE") {
                sec = OBJSENSE;
                if (t.size() > 1) {
                    const std::string v = upper(t[1]);
                    if (v == "MAX" || v == "MAXIMIZE") sense = DLP_MAXIMIZE;
                    else if (v == "MIN" || v == "MINIMIZE") sense = DLP_MINIMIZE;
                    else fail("bad OBJSENSE " + t[1]);
                }
            } else {
                fail("unknown section " + t[0]);
            }
            continue;
        }
        switch (sec) {
            case OBJSENSE: {
                const std::string v = upper(t[0]);
                if (v == "MAX" || v == "MAXIMIZE") sense = DLP_MAXIMIZE;
                else if (v == "MIN" || v == "MINIMIZE") sense = DLP_MINIMIZE;
                else fail("bad OBJSENSE " + t[0]);
                break;
            }
            case ROWS: {
                if (t.size() != 2) { fail("ROWS needs: type name"); break; }
                const std::string ty = upper(t[0]);
                if (row_id.count(t[1])) { fail("duplicate row " + t[1]); break; }
                if (ty == "N") {
                    if (objname.empty()) { objname = t[1]; row_id[t[1]] = -1; }
                    else row_id[t[1]] = -2;
                } else if (ty == "L" || ty == "G" || ty == "E") {
                    row_id[t[1]] = (int64_t)rtype.size();
                    rtype.push_back(ty[0]);
                    rhs.push_back(0.0);
                    range.push_back(0.0);
                    has_range.push_back(false);
                } else {
                    fail("bad row type " + t[0]);
                }
                break;
            }
            case COLUMNS: {
                if (t.size() >= 2 && t[1] == "'MARKER'") break;   // integrality markers: LP relaxation
                if (t.size() != 3 && t.size() != 5) { fail("COLUMNS needs: col row value [row value]"); break; }
                int64_t j;
                auto it = col_id.find(t[0]);
                if (it == col_id.end()) {
                    j = (int64_t)c.size();
                    col_id[t[0]] = j;
                    c.push_back(0.0);
                    lo.push_back(0.0);
                    hi.push_back(HUGE_VAL);
                } else {
                    j = it->second;
                }
                for (size_t k = 1; k + 1 < t.size(); k += 2) {
                    int64_t i;
                    double v;
                    if (!row_of(t[k], &i)) break;
                    if (!number(t[k + 1], &v)) { fail("bad number " + t[k + 1]); break; }
                    if (i == -1) c[j] += v;
                    else if (i >= 0) entries.push_back({i, j, v});
                }
                break;
            }
            case RHS:
            case RANGES: {
                const size_t k0 = (t.size() % 2 == 1) ? 1 : 0;   // optional set name
                if (t.size() < 2 || t.size() > 5) { fail("RHS/RANGES needs: [set] row value [row value]"); break; }
                for (size_t k = k0; k + 1 < t.size(); k += 2) {
                    int64_t i;
                    double v;
                    if (!row_of(t[k], &i)) break;
                    if (!number(t[k + 1], &v)) { fail("bad number " + t[k + 1]); break; }
                    if (sec == RHS) {
                        if (i == -1) c0 = -v;
                        else if (i >= 0) rhs[i] = v;
                    } else if (i >= 0) {
                        range[i] = v;
                        has_range[i] = true;
                    }
                }
                break;
            }
            case BOUNDS: {
                if (t.size() < 2) { fail("BOUNDS needs: type [set] col [value]"); break; }
                const std::string ty = upper(t[0]);
                const bool valued = ty == "UP" || ty == "LO" || ty == "FX" || ty == "LI" || ty == "UI";
                const bool novalue = ty == "FR" || ty == "MI" || ty == "PL" || ty == "BV";
                if (!valued && !novalue) { fail("unsupported bound type " + t[0]); break; }
                // field layout: type [set] col [value]; the set name is optional
                size_t kc;
                double probe;
                if (valued) {
                    if (t.size() == 4) kc = 2;
                    else if (t.size() == 3) kc = 1;
                    else { fail("bound needs a value"); break; }
                } else if (t.size() == 2) {
                    kc = 1;
                } else if (t.size() == 3) {   // "type set col", or "BV col value"
                    kc = (col_id.count(t[1]) && number(t[2], &probe)) ? 1 : 2;
                } else if (t.size() == 4) {   // "BV set col value"
                    kc = 2;
                } else {
                    fail("bad BOUNDS line");
                    break;
                }
                int64_t j;
                if (!col_of(t[kc], &j)) break;
                double v = 0.0;
                if (valued && !number(t[kc + 1], &v)) { fail("bad number " + t[kc + 1]); break; }
                if (ty == "UP" || ty == "UI") {
                    hi[j] = v;
                    if (v < 0.0 && lo[j] == 0.0) lo[j] = -HUGE_VAL;
                } else if (ty == "LO" || ty == "LI") {
                    lo[j] = v;
                } else if (ty == "FX") {
                    lo[j] = v;
                    hi[j] = v;
                } else if (ty == "FR") {
                    lo[j] = -HUGE_VAL;
                    hi[j] = HUGE_VAL;
                } else if (ty == "MI") {
                    lo[j] = -HUGE_VAL;
                } else if (ty == "PL") {
                    hi[j] = HUGE_VAL;
                } else {   // BV
                    lo[j] = 0.0;
                    hi[j] = 1.0;
                }
                break;
            }
            case NAME:
            case NONE:
            default:
                fail("data line outside a section");
                break;
        }
    }
    std::fclose(f);
    if (err.empty() && sec != END) fail("missing ENDATA");
    if (err.empty() && objname.empty()) fail("no objective (N) row");
    if (!err.empty()) {
        set_error(err);
        return DLP_ERR_ARG;
    }
    General& g = *out;
    g = General();
    g.m = (int64_t)rtype.size();
    g.n = (int64_t)c.size();
    if (g.n == 0) {
        set_error("MPS file has no columns");
        return DLP_ERR_ARG;
    }
    g.A.assign((size_t)g.m * g.n, 0.0);
    for (const Entry& e : entries) g.A[e.i * g.n + e.j] += e.v;   // repeated entries are summed
    g.row_lo.resize(g.m);
    g.row_hi.resize(g.m);
    for (int64_t i = 0; i < g.m; ++i) {
        const double b = rhs[i], r = std::fabs(range[i]);
        switch (rtype[i]) {
            case 'L': g.row_lo[i] = has_range[i] ? b - r : -HUGE_VAL; g.row_hi[i] = b; break;
            case 'G': g.row_lo[i] = b; g.row_hi[i] = has_range[i] ? b + r : HUGE_VAL; break;
            default:   // E
                g.row_lo[i] = b;
                g.row_hi[i] = b;
                if (has_range[i] && range[i] > 0) g.row_hi[i] = b + r;
                if (has_range[i] && range[i] < 0) g.row_lo[i] = b - r;
                break;
        }
    }
    g.col_lo = lo;
    g.col_hi = hi;
    g.c = c;
    g.c0 = c0;
    g.sense = sense;
    return DLP_OK;
}

}  // namespace dlp
