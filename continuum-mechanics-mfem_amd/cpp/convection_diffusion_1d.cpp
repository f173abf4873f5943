// convection_diffusion_1d — the reference's transient three-Peclet convection-diffusion driver
// (myapps/convection_diffusion/linear_convection_diffusion_1D.cpp) through the MFEM-shaped host API,
// every operator resident on the GPU across time steps, one MPI rank per GPU.
//
// Despite its name the reference problem is quasi-1D on the 2D unit square: c_t + c_x = c_xx / Pe,
// Dirichlet on the x-extremes (BuildXDirichletBoundaryMarker, :219-266), natural Neumann on y, so
// the solution is the 1D erfc profile (:128-166) in every y.  Backward Euler, three uncoupled
// systems (Pe = 1, 10, 100): (M + dt C(beta) + (dt/Pe) K) c^{n+1} = M c^n (:375-400), each step
// rhs_k = M c_k (mass_form.Mult), ProjectBdrCoefficient, FormLinearSystem, PETSc solve per block,
// RecoverFEMSolution, and the L2 error of each block against its exact solution (:483-510, 537-576).
// The call forms are the reference's; configuration comes from the command line instead of YAML
// and the ParaView output is omitted (the error history CSV is kept, same columns).
//
//   mpirun -np N convection_diffusion_1d [-mesh file.msh | -n elems] [-p order] [-rs l] [-rp l]
//        [-dt dt] [-T t_final] [-pe1 1] [-pe2 10] [-pe3 100] [-opts petsc.opts] [-csv file]
// Output (rank 0): dofs, ranks, steps, abs_l2_pe{1,2,3}, rel_l2_pe{1,2,3} at the final step,
// gmres_iterations, seconds_per_step.  Exit code 3 on error.
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iomanip>
#include <limits>
#include <memory>
#include <string>

#include "mfem.hpp"

using namespace std;
using namespace mfem;

namespace {


// exp(a) erfc(b) without inf * 0 for large b (:128-144): the asymptotic erfc series past b = 26
double ExpTimesErfc(const double a, const double b)
{
    if (b > 26.0) {
        const double ib = 1.0 / b, ib2 = ib * ib;
        const double erfc_asym = ib / std::sqrt(M_PI) * (1.0 - 0.5 * ib2 + 0.75 * ib2 * ib2);
        const double expo = a - b * b;
        if (expo < -745.0) return 0.0;
        if (expo > 709.0) return numeric_limits<double>::infinity();
        return std::exp(expo) * erfc_asym;
    }
    if (a > 709.0) return numeric_limits<double>::infinity();
    return std::exp(a) * std::erfc(b);
}

// the 1D solution of c_t + c_x = c_xx / Pe on x > 0, c(0, t) = 1, c(x, 0) = 0 (:146-166)
double ExactConcentration(const double x, const double t, const double pe)
{
    if (t <= 0.0) return 0.0;
    const double diff = t / pe, root = std::sqrt(diff);
    const double arg1 = (x - t) / (2.0 * root), arg2 = (x + t) / (2.0 * root);
    const double gauss = -((x - t) * (x - t)) / (4.0 * diff);
    const double c = 0.5 * std::erfc(arg1) + std::sqrt(t * pe / M_PI) * std::exp(gauss) -
                     0.5 * (1.0 + pe * x + pe * t) * ExpTimesErfc(pe * x, arg2);
    return std::isfinite(c) ? c : 0.0;
}

class ExactConcentrationCoefficient : public Coefficient {
public:
    explicit ExactConcentrationCoefficient(double pe) : pe_(pe) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        return ExactConcentration(x[0], GetTime(), pe_);
    }

private:
    double pe_;
};

void ValidateUnitSquareMesh(const ParMesh &pmesh, const double tol)  // :168-195
{
    double lmin[2] = {numeric_limits<double>::infinity(), numeric_limits<double>::infinity()};
    double lmax[2] = {-numeric_limits<double>::infinity(), -numeric_limits<double>::infinity()};
    for (int i = 0; i < pmesh.GetNV(); i++) {
        const double *v = pmesh.GetVertex(i);
        for (int k = 0; k < 2; k++) {
            lmin[k] = std::min(lmin[k], v[k]);
            lmax[k] = std::max(lmax[k], v[k]);
        }
    }
    double gmin[2] = {0.0, 0.0}, gmax[2] = {0.0, 0.0};
    MPI_Allreduce(lmin, gmin, 2, MPI_DOUBLE, MPI_MIN, MPI_COMM_WORLD);
    MPI_Allreduce(lmax, gmax, 2, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    MFEM_VERIFY(std::abs(gmin[0]) <= tol && std::abs(gmax[0] - 1.0) <= tol && std::abs(gmin[1]) <= tol &&
                    std::abs(gmax[1] - 1.0) <= tol,
                "Mesh coordinates must span approximately [0,1]x[0,1]. Got x=[" << gmin[0] << "," << gmax[0]
                                                                                << "], y=[" << gmin[1] << ","
                                                                                << gmax[1] << "].");
}

// boundary attributes whose elements' centres lie on x = xmin or x = xmax (:219-266)
void BuildXDirichletBoundaryMarker(ParMesh &pmesh, Array<int> &ess_bdr, const double tol)
{
    const int nbdr = pmesh.bdr_attributes.Max();
    MFEM_VERIFY(nbdr > 0, "Mesh must define boundary attributes.");
    double lxmin = numeric_limits<double>::infinity(), lxmax = -numeric_limits<double>::infinity();
    for (int i = 0; i < pmesh.GetNV(); i++) {
        const double *v = pmesh.GetVertex(i);
        lxmin = std::min(lxmin, v[0]);
        lxmax = std::max(lxmax, v[0]);
    }
    double xmin = 0.0, xmax = 0.0;
    MPI_Allreduce(&lxmin, &xmin, 1, MPI_DOUBLE, MPI_MIN, MPI_COMM_WORLD);
    MPI_Allreduce(&lxmax, &xmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    ess_bdr.SetSize(nbdr);
    ess_bdr = 0;
    Vector x;
    for (int i = 0; i < pmesh.GetNBE(); i++) {
        const int attr = pmesh.GetBdrAttribute(i);
        ElementTransformation *T = pmesh.GetBdrElementTransformation(i);
        const IntegrationPoint &ip = Geometries.GetCenter(T->GetGeometryType());
        T->Transform(ip, x);
        if (std::abs(x[0] - xmin) <= tol || std::abs(x[0] - xmax) <= tol) ess_bdr[attr - 1] = 1;
    }
    Array<int> global_marker(nbdr);
    global_marker = 0;
    MPI_Allreduce(ess_bdr.GetData(), global_marker.GetData(), nbdr, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    ess_bdr = global_marker;
    int count = 0;
    for (int a = 0; a < nbdr; a++) count += ess_bdr[a];
    MFEM_VERIFY(count > 0, "Failed to identify Dirichlet boundaries at x-extremes.");
}

}  // namespace

int main(int argc, char *argv[])
{
    Mpi::Init(argc, argv);
    Hypre::Init();
    const int myid = Mpi::WorldRank();

    string mesh_file, opts, csv;
    int n = 32, order = 3, rs = 0, rp = 0;
    double dt = 1.0e-3, t_final = 1.0;  // Input/input.yaml
    array<double, 3> peclet = {1.0, 10.0, 100.0};
    OptionsParser args(argc, argv);
    args.AddOption(&mesh_file, "-mesh", "--mesh", "gmsh v2.2 mesh file (else a Cartesian square).");
    args.AddOption(&n, "-n", "--elems", "Elements per direction of the generated square.");
    args.AddOption(&order, "-p", "--order", "H1 order.");
    args.AddOption(&rs, "-rs", "--serial-ref-levels", "Uniform refinements before the partition.");
    args.AddOption(&rp, "-rp", "--par-ref-levels", "Uniform refinements after the partition.");
    args.AddOption(&dt, "-dt", "--dt", "Time step.");
    args.AddOption(&t_final, "-T", "--t-final", "Final time.");
    args.AddOption(&peclet[0], "-pe1", "--peclet1", "Peclet number of system 1.");
    args.AddOption(&peclet[1], "-pe2", "--peclet2", "Peclet number of system 2.");
    args.AddOption(&peclet[2], "-pe3", "--peclet3", "Peclet number of system 3.");
    args.AddOption(&opts, "-opts", "--petsc-options", "PETSc options file.");
    args.AddOption(&csv, "-csv", "--error-csv", "Error history CSV (rank 0; empty: none).");
    args.Parse();
    if (!args.Good()) {
        if (myid == 0) args.PrintUsage(cerr);
        return 1;
    }
    if (order < 1 || dt <= 0.0 || t_final < 0.0 || peclet[0] <= 0.0 || peclet[1] <= 0.0 || peclet[2] <= 0.0) {
        if (myid == 0) cerr << "Error: order >= 1, dt > 0, t_final >= 0 and Peclet > 0 required (:103-125)" << endl;
        return 2;
    }
    const char *petsc_file_to_use = DriverPetscOptionsFile(opts);
    MFEMInitializePetsc(&argc, &argv, petsc_file_to_use, NULL);

    int exit_code = 0;
    try {
        Device device("cpu");

        unique_ptr<Mesh> mesh = mesh_file.empty()
                                    ? make_unique<Mesh>(Mesh::MakeCartesian2D(n, n, Element::QUADRILATERAL))
                                    : make_unique<Mesh>(mesh_file.c_str(), 1, 1);
        if (mesh->Dimension() != 2) throw runtime_error("The mesh must be 2D.");
        for (int l = 0; l < rs; l++) mesh->UniformRefinement();
        unique_ptr<ParMesh> pmesh = make_unique<ParMesh>(MPI_COMM_WORLD, *mesh);
        mesh.reset();
        for (int l = 0; l < rp; l++) pmesh->UniformRefinement();
        MFEM_VERIFY(pmesh->bdr_attributes.Size() > 0, "Mesh must define boundary attributes.");
        ValidateUnitSquareMesh(*pmesh, 1.0e-8);

        H1_FECollection fec(order, 2);
        ParFiniteElementSpace fespace(pmesh.get(), &fec);
        const HYPRE_BigInt global_true_dofs = fespace.GlobalTrueVSize();

        Array<int> ess_bdr;
        BuildXDirichletBoundaryMarker(*pmesh, ess_bdr, 1.0e-8);
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ParBilinearForm mass_form(&fespace);  // :375-378
        mass_form.AddDomainIntegrator(new MassIntegrator());
        mass_form.Assemble();
        mass_form.Finalize();

        Vector beta_vec(2);  // :380-383
        beta_vec = 0.0;
        beta_vec[0] = 1.0;
        VectorConstantCoefficient beta_coeff(beta_vec);
        array<ConstantCoefficient, 3> diffusion_coeff = {ConstantCoefficient(dt / peclet[0]),
                                                         ConstantCoefficient(dt / peclet[1]),
                                                         ConstantCoefficient(dt / peclet[2])};
        array<unique_ptr<ParBilinearForm>, 3> forms;  // :391-400
        for (int k = 0; k < 3; k++) {
            forms[k] = make_unique<ParBilinearForm>(&fespace);
            forms[k]->AddDomainIntegrator(new MassIntegrator());
            forms[k]->AddDomainIntegrator(new ConvectionIntegrator(beta_coeff, dt));
            forms[k]->AddDomainIntegrator(new DiffusionIntegrator(diffusion_coeff[k]));
            forms[k]->Assemble();
            forms[k]->Finalize();
        }
        array<unique_ptr<ParGridFunction>, 3> c;
        for (int k = 0; k < 3; k++) {
            c[k] = make_unique<ParGridFunction>(&fespace);
            *(c[k]) = 0.0;
        }
        array<ExactConcentrationCoefficient, 3> exact_coeffs = {ExactConcentrationCoefficient(peclet[0]),
                                                                ExactConcentrationCoefficient(peclet[1]),
                                                                ExactConcentrationCoefficient(peclet[2])};
        const int true_size = fespace.TrueVSize();
        const bool all_essential = (ess_tdof_list.Size() == true_size);
        array<Vector, 3> rhs_local, X_sub, B_sub;
        array<OperatorHandle, 3> Ah = {OperatorHandle(Operator::Hypre_ParCSR), OperatorHandle(Operator::Hypre_ParCSR),
                                       OperatorHandle(Operator::Hypre_ParCSR)};
        const int nsteps = static_cast<int>(std::ceil(t_final / dt - 1.0e-12));

        ofstream err_csv;
        if (myid == 0 && !csv.empty()) {
            err_csv.open(csv);
            if (!err_csv) throw runtime_error("Failed to open error CSV: " + csv);
            err_csv << "step,time,abs_l2_pe1,rel_l2_pe1,abs_l2_pe2,rel_l2_pe2,abs_l2_pe3,rel_l2_pe3\n"
                    << setprecision(16);
        }
        const int order_quad = std::max(2, 2 * order + 3);  // :483-488
        const IntegrationRule *irs[Geometry::NumGeom];
        for (int g = 0; g < Geometry::NumGeom; g++) irs[g] = &IntRules.Get(g, order_quad);
        array<double, 3> abs_l2 = {0.0, 0.0, 0.0}, rel_l2 = {0.0, 0.0, 0.0};
        auto write_errors = [&](int step, double t) {  // :490-522 (collective)
            for (int k = 0; k < 3; k++) {
                exact_coeffs[k].SetTime(t);
                abs_l2[k] = c[k]->ComputeL2Error(exact_coeffs[k], irs);
                const double norm_l2 = ComputeGlobalLpNorm(2, exact_coeffs[k], *pmesh, irs);
                rel_l2[k] = (norm_l2 > 1.0e-14) ? abs_l2[k] / norm_l2 : 0.0;
            }
            if (myid == 0 && err_csv.is_open())
                err_csv << step << "," << t << "," << abs_l2[0] << "," << rel_l2[0] << "," << abs_l2[1] << ","
                        << rel_l2[1] << "," << abs_l2[2] << "," << rel_l2[2] << "\n";
        };
        write_errors(0, 0.0);

        long gmres_its = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int step = 1; step <= nsteps; step++) {  // :537-576
            const double t = step * dt;
            for (int k = 0; k < 3; k++) {
                rhs_local[k].SetSize(fespace.GetVSize());
                mass_form.Mult(*(c[k]), rhs_local[k]);
                exact_coeffs[k].SetTime(t);
                c[k]->ProjectBdrCoefficient(exact_coeffs[k], ess_bdr);
                forms[k]->FormLinearSystem(ess_tdof_list, *(c[k]), rhs_local[k], Ah[k], X_sub[k], B_sub[k]);
            }
            if (!all_essential) {
                for (int k = 0; k < 3; k++) {
                    HypreParMatrix *Ak = Ah[k].As<HypreParMatrix>();
                    MFEM_VERIFY(Ak != nullptr, "Expected HypreParMatrix in block " << k);
                    PetscParMatrix A_petsc(Ak, Operator::PETSC_MATAIJ);
                    PetscLinearSolver solver(A_petsc);
                    solver.SetPrintLevel(0);
                    solver.Mult(B_sub[k], X_sub[k]);
                    MFEM_VERIFY(solver.GetConverged(), "PETSc solver did not converge at step "
                                                           << step << ", block " << k << ". Iterations="
                                                           << solver.GetNumIterations()
                                                           << ", residual=" << solver.GetFinalNorm());
                    gmres_its += solver.GetNumIterations();
                }
            }
            for (int k = 0; k < 3; k++) forms[k]->RecoverFEMSolution(X_sub[k], rhs_local[k], *(c[k]));
            write_errors(step, t);
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (myid == 0)
            std::printf("dofs %lld\nranks %d\nsteps %d\nabs_l2_pe1 %.17g\nabs_l2_pe2 %.17g\nabs_l2_pe3 %.17g\n"
                        "rel_l2_pe1 %.17g\nrel_l2_pe2 %.17g\nrel_l2_pe3 %.17g\ngmres_iterations %ld\n"
                        "seconds_per_step %.6g\n",
                        (long long)global_true_dofs, Mpi::WorldSize(), nsteps, abs_l2[0], abs_l2[1], abs_l2[2],
                        rel_l2[0], rel_l2[1], rel_l2[2], gmres_its, secs / std::max(nsteps, 1));
    } catch (const exception &e) {
        if (myid == 0) cerr << "Error: " << e.what() << endl;
        exit_code = 3;
    }

    MFEMFinalizePetsc();
    return exit_code;
}
