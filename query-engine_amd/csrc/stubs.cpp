// Temporary entry points for operators whose kernels are still being written.
#include "qeh_internal.h"
using namespace qeh;
extern "C" {
int qeh_filter(qeh_ctx *, const qeh_column *, int, const qeh_expr *, const int32_t *, int, qeh_column *, int64_t *) { return fail(QEH_E_UNSUPPORTED, "qeh_filter: not built yet"); }
int qeh_eval(qeh_ctx *, const qeh_column *, int, const qeh_expr *, int64_t, qeh_column *) { return fail(QEH_E_UNSUPPORTED, "qeh_eval: not built yet"); }
int qeh_hash_join_inner(qeh_ctx *, const qeh_column *, const qeh_column *, int, const qeh_column *, const qeh_column *, int, qeh_column *, qeh_column *, int64_t *) { return fail(QEH_E_UNSUPPORTED, "not built yet"); }
int qeh_sort_indices(qeh_ctx *, const qeh_column *, int, const int8_t *, qeh_column *) { return fail(QEH_E_UNSUPPORTED, "not built yet"); }
int qeh_take(qeh_ctx *, const qeh_column *, const qeh_column *, qeh_column *) { return fail(QEH_E_UNSUPPORTED, "not built yet"); }
int qeh_row_number(qeh_ctx *, const qeh_column *, int, const qeh_column *, int, const int8_t *, qeh_column *) { return fail(QEH_E_UNSUPPORTED, "not built yet"); }
int qeh_hash_partition(qeh_ctx *, const qeh_column *, int, int64_t *, qeh_column *) { return fail(QEH_E_UNSUPPORTED, "not built yet"); }
}
