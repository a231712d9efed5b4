"""Reporting helpers (N9): the reference's two regression plots (ref.py:201-223) rendered
headless with ``savefig`` (its ``plt.show()`` blocks or no-ops on a cluster driver, D10),
and the operational-insights report (ref.py:245-255)."""
from __future__ import annotations

import os
from typing import Dict, Optional


def regression_plots(predictions_pd, out_dir: str, model_name: str = "Linear Regression",
                     label: str = "length_of_stay", prediction: str = "prediction") -> Dict[str, str]:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    os.makedirs(out_dir, exist_ok=True)
    pdf = predictions_pd
    if "residual" not in pdf.columns:
        pdf = pdf.assign(residual=pdf[label] - pdf[prediction])
    paths = {}
    fig = plt.figure(figsize=(8, 6))
    plt.scatter(pdf[label], pdf[prediction], alpha=0.6, color="blue")
    plt.xlabel("Actual Length of Stay")
    plt.ylabel("Predicted Length of Stay")
    plt.title(f"Predicted vs. Actual Length of Stay ({model_name})")
    lo, hi = pdf[label].min(), pdf[label].max()
    plt.plot([lo, hi], [lo, hi], color="red", lw=2)
    paths["pred_vs_actual"] = os.path.join(out_dir, "pred_vs_actual.png")
    fig.savefig(paths["pred_vs_actual"])
    plt.close(fig)
    fig = plt.figure(figsize=(8, 6))
    plt.scatter(pdf[prediction], pdf["residual"], alpha=0.6, color="green")
    plt.xlabel("Predicted Length of Stay")
    plt.ylabel("Residuals (Actual - Predicted)")
    plt.title(f"Residual Plot ({model_name})")
    plt.axhline(y=0, color="red", linestyle="--")
    paths["residuals"] = os.path.join(out_dir, "residuals.png")
    fig.savefig(paths["residuals"])
    plt.close(fig)
    return paths


def operational_insights(lr_rmse: float, dt_rmse: float, rf_rmse: float, dt_acc: float, rf_acc: float) -> str:
    lines = [
        "",
        "--- Operational Insights ---",
        "Analysis indicates that high admission counts, increased emergency visits, and seasonal trends",
        "correlate with longer patient lengths of stay. The regression models provide RMSE values as follows:",
        f"Linear Regression RMSE: {lr_rmse}",
        f"Decision Tree Regression RMSE: {dt_rmse}",
        f"Random Forest Regression RMSE: {rf_rmse}",
        "For classification (high vs. low LOS), accuracies are:",
        f"Decision Tree Classifier Accuracy: {dt_acc}",
        f"Random Forest Classifier Accuracy: {rf_acc}",
        "Recommendations: Adjust staffing and optimize discharge procedures during peak times to reduce LOS.",
        "----------------------------",
    ]
    return "\n".join(lines)
