"""The reference's seed deck (app.mjs:188-224): Jessica plus test cards t1..t11.

Used by the trait-card model (:mod:`mikmeans.models.room`) and as the
dashboard-parity fixture.  Fixed ids ``seed:jessica``,
``seed:t1`` .. ``seed:t11``; t10/t11 are the labelled outliers (app.mjs:214-215).
"""
from __future__ import annotations

JESSICA = {"id": "seed:jessica", "title": "Jessica", "traits": ["Fresh", "Sorbet"]}

TEST_ITEMS = [
    ("seed:t1", "Nguyen", "Sweet", "Creamy"),
    ("seed:t2", "Patel", "Fresh", "Sorbet"),
    ("seed:t3", "Garcia", "Chocolatey", "Crunchy"),
    ("seed:t4", "Rossi", "Milky", "Silky"),
    ("seed:t5", "Kim", "Nutty", "Creamy"),
    ("seed:t6", "Smith", "Fruity", "Swirled"),
    ("seed:t7", "Ahmed", "Bitter", "Rich"),
    ("seed:t8", "Lopez", "Sweet", "Colorful"),
    ("seed:t9", "Chen", "Rich", "Spicy"),
    ("seed:t10", "Nils", "Espresso", "Hot"),      # outlier
    ("seed:t11", "sally", "Vegan", "Not Sweet"),  # outlier
]


def demo_cards(assigned_to=None) -> list[dict]:
    """Jessica + t1..t11 as card records ``{id, title, traits, assignedTo, createdBy}``."""
    cards = [{"id": JESSICA["id"], "title": JESSICA["title"], "traits": list(JESSICA["traits"]),
              "assignedTo": None, "createdBy": "seed"}]
    for cid, title, a, b in TEST_ITEMS:
        cards.append({"id": cid, "title": title, "traits": [a, b], "assignedTo": None, "createdBy": "seed"})
    if assigned_to:
        for c in cards:
            c["assignedTo"] = assigned_to.get(c["id"])
    return cards
