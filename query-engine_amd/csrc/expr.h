// Expression programs: the host compiles a postfix `PhysicalExpr`
// (qeh_expr, include/qeh.h) into a typed register program that every kernel
// interprets with wave-uniform dispatch.  Typing / coercion follows the
// reference exactly (operators.rs:382-709); errors carry the reference's text.
#pragma once

#include <stdint.h>

#include "../../include/qeh.h"
#include "device_common.h"

namespace qeh {

constexpr int kNS = 8;        // value slots (= max stack depth)
constexpr int kMaxInstr = 40;

enum DevOp : uint8_t {
    D_LOAD = 0,   // dst <- column[a]            (t = column dtype)
    D_LIT,        // dst <- imm / NULL           (t = dtype, flag = is_null)
    D_TOF64,      // dst <- (double) int slot a  (t = source dtype)
    D_ADD, D_SUB, D_MUL, D_DIV, D_MOD,         // t = operand dtype
    D_EQ, D_NE, D_LT, D_LE, D_GT, D_GE,        // t = operand dtype (after coercion)
    D_AND, D_OR, D_NOT, D_NEG
};

struct DevInstr {
    uint8_t op, t, dst, a;
    uint8_t b, flag, pad0, pad1;
    int64_t imm;
};

struct DevProgram {
    int32_t n;            // instructions
    int32_t result_type;  // dtype of slot 0 after the program
    DevInstr ins[kMaxInstr];
};

// Fast path: a single-level AND-list or OR-list of `column CMP literal`
// comparisons (the shape of every predicate in the BASELINE configs).
constexpr int kMaxTerms = 6;
struct PredTerm {
    int32_t col;      // column index
    int32_t ctype;    // compare type: QEH_DT_INT64 or QEH_DT_FLOAT64 (or BOOL)
    int32_t op;       // D_EQ..D_GE with the column on the left
    int32_t _pad;
    int64_t lit;      // int64 literal, or totalOrder key of the double literal
};
struct PredTerms {
    int32_t n;        // 0 = always TRUE (no predicate)
    int32_t is_or;    // 0 = AND-list, 1 = OR-list (non-Kleene, arrow and/or)
    PredTerm t[kMaxTerms];
};

// error bits reported by kernels (atomicOr into a scratch word)
constexpr uint32_t kErrOverflow = 1u;
constexpr uint32_t kErrDiv0 = 2u;
constexpr uint32_t kErrModOverflow = 4u;
constexpr uint32_t kErrSpin = 8u;

// Host side --------------------------------------------------------------------
// Compile `e` over columns of `dtypes`.  Returns QEH_OK or an error status with
// qeh_last_error set to the reference's message.
int compile_expr(const qeh_expr *e, const int32_t *dtypes, int n_cols, DevProgram *out);
// Try to lower to the fast term list (only for BOOL-typed predicates).
bool lower_to_terms(const qeh_expr *e, const int32_t *dtypes, int n_cols, PredTerms *out);
// Index of the column a bare Column expression refers to, else -1.
int expr_as_column(const qeh_expr *e);
// Columns referenced by an expression (bitmask over <= 64 columns).
uint64_t expr_columns(const qeh_expr *e);

}  // namespace qeh
