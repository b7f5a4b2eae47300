from .elicitation import (  # noqa: F401
    WORD_PLURALS,
    accuracy,
    any_pass_at_k,
    calculate_metrics,
    delta_nll,
    global_majority_vote_at_k,
    id_topk_scores,
    leak_rate,
    majority_at_k,
    pass_at_k,
    prompt_accuracy_at_k,
    word_metrics,
)
from .bootstrap import bootstrap_ci, grouped_bootstrap_ci, summarize  # noqa: F401
