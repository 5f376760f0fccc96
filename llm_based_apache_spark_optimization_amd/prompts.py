"""Prompt contracts of the reference, kept byte-compatible.

* NL->SQL (LLM#1, model ``duckdb-nsql``): FastAPI/app.py:79,85-89 and Flask/app.py:98,102-106.
* Spark-error explanation (LLM#2, model ``llama3.2``): FastAPI/app.py:99-111, Flask/app.py:153-166.
* Evaluation-harness prompts: Model_Evaluation_&_Comparision.py:8-16,25-39,86-103,116.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

NL2SQL_MODEL = "duckdb-nsql"
EXPLAIN_MODEL = "llama3.2"

EXPLAIN_SYSTEM = "You are an AI that helps troubleshoot Apache Spark errors. Provide clear, concise solutions."


def table_schema_text(dtypes: Iterable[Tuple[str, str]]) -> str:
    """``"\\n".join(f"{col} ({dtype})" for col, dtype in df.dtypes)`` with Spark type strings."""
    return "\n".join([f"{col} ({dtype})" for col, dtype in dtypes])


def nl2sql_system(table_schema: str) -> str:
    return f"Table name is temp_view. The structure of the table is:\n{table_schema}"


def explain_prompt(error_message: str) -> str:
    return (
        f"The following Spark error occurred:\n\n"
        f"{error_message}\n\n"
        f"Please analyze this error and suggest possible solutions."
    )


# ------------------------------------------------------------------ evaluation harness (C21/C22/C26)
EVAL_EXPECTED_SQL = (
    "SELECT VendorID, \n"
    "       SUM(total_amount) AS total_fare, \n"
    "       AVG(trip_distance) AS avg_trip_distance\n"
    "FROM taxi\n"
    "WHERE passenger_count > 2\n"
    "GROUP BY VendorID\n"
    "ORDER BY total_fare DESC;"
)

EVAL_SINGLE_SYSTEM = (
    "Here is the database schema that the SQL query will run on: \n"
    "        CREATE TABLE taxi (\n"
    "            VendorID bigint, \n"
    "            tpep_pickup_datetime timestamp, \n"
    "            tpep_dropoff_datetime timestamp, \n"
    "            passenger_count double, \n"
    "            trip_distance double, \n"
    "            fare_amount double, \n"
    "            extra double, \n"
    "            tip_amount double, \n"
    "            tolls_amount double, \n"
    "            improvement_surcharge double, \n"
    "            total_amount double\n"
    "        );"
)

EVAL_SINGLE_PROMPT = (
    "Provide me with the total fare amount, including tips and tolls, for each vendor, along with the average "
    "trip distance, for trips that had more than 2 passengers, sorted by total fare amount in descending order?"
)

EVAL_MULTI_SYSTEM = (
    "Here is the database schema that the SQL query will run on: CREATE TABLE taxi (VendorID bigint, "
    "tpep_pickup_datetime timestamp, tpep_dropoff_datetime timestamp, passenger_count double, trip_distance "
    "double, fare_amount double, extra double, tip_amount double, tolls_amount double, improvement_surcharge "
    "double, total_amount double,);"
)

EVAL_QUERIES: Sequence[dict] = (
    {"nl": "Get all taxis with more than 2 passengers.",
     "expected_sql": "SELECT * FROM taxi WHERE passenger_count > 2;"},
    {"nl": "Show total fare collected by each vendor.",
     "expected_sql": "SELECT VendorID, SUM(total_amount) AS Total_Fare FROM taxi GROUP BY VendorID;"},
    {"nl": "Find the average trip distance for trips that had more than 2 passengers.",
     "expected_sql": "SELECT AVG(trip_distance) FROM taxi WHERE passenger_count > 2;"},
    {"nl": "List all vendors ordered by total fare in descending order.",
     "expected_sql": "SELECT VendorID, SUM(total_amount) AS Total_Fare FROM taxi GROUP BY VendorID ORDER BY "
                     "Total_Fare DESC;"},
)

EVAL_MODELS = ("mistral", "llama3.2", "duckdb-nsql")
