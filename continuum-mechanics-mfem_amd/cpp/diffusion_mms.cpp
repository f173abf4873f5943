// diffusion_mms — transient diffusion MMS with backward Euler through the MFEM-shaped host API,
// operators resident on the GPU across time steps, one MPI rank per GPU.
//
// The time loop is the reference's, myapps/convection_diffusion/diffusion_mms.cpp:238-483, with its
// call forms unchanged: Mpi::Init, Device("cpu"), make_unique<ParMesh>(MPI_COMM_WORLD, *mesh), mass
// and LHS forms (M and M + alpha dt K) assembled once (:294-305); per step rhs = M u_old
// (mass_form.Mult, a rank-local partial vector, :430), rhs += dt (f(t), v) (:433-437),
// ProjectBdrCoefficient (:440-441), FormLinearSystem (:444), PetscParMatrix(A_hyp, PETSC_MATAIJ) +
// PetscLinearSolver (:447-456), MFEM_VERIFY(GetConverged), RecoverFEMSolution (:459); L2 and
// MPI-reduced Linf errors (:367-383).  Exact u = sin(t) cos(2(x-1/2)^2 + 2(y-1/2)^2),
// f = u_t - alpha Lap u (:136-178).  On the GPU both operators stay resident; FormLinearSystem per
// step is B = P^T(b - A x_e), B_ess = x_ess on the already-eliminated operator (no re-assembly, no RAP
// as hypre does at :444).  Configuration from the command line instead of YAML; no ParaView / CSV.
//
//   mpirun -np N diffusion_mms [-mesh file.msh | -n elems] [-p order] [-rs l] [-rp l] [-a alpha]
//                              [-dt dt] [-T t_final] [-opts petsc.opts]
// Output (rank 0): dofs, ranks, steps, final_l2, final_linf, gmres_iterations, seconds_per_step.
// Exit code 3 on error.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <memory>
#include <string>

#include "mfem.hpp"

using namespace std;
using namespace mfem;

namespace {


class ExactCoefficient : public Coefficient {
public:
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const double dx = x[0] - 0.5, dy = x[1] - 0.5;
        return std::sin(GetTime()) * std::cos(2.0 * dx * dx + 2.0 * dy * dy);
    }
};

class ForcingCoefficient : public Coefficient {
public:
    explicit ForcingCoefficient(double alpha) : alpha_(alpha) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const double t = GetTime(), dx = x[0] - 0.5, dy = x[1] - 0.5;
        const double r2 = dx * dx + dy * dy, q = 2.0 * r2;
        const double ut = std::cos(t) * std::cos(q);
        const double lap = std::sin(t) * (-16.0 * r2 * std::cos(q) - 8.0 * std::sin(q));
        return ut - alpha_ * lap;
    }

private:
    double alpha_;
};

}  // namespace

int main(int argc, char *argv[])
{
    Mpi::Init(argc, argv);
    Hypre::Init();
    const int myid = Mpi::WorldRank();

    string mesh_file, opts;
    int n = 16, order = 1, rs = 0, rp = 0;
    double alpha = 0.1, dt = 0.05, t_final = 2.0;  // Input/input_diffusion_mms.yaml
    OptionsParser args(argc, argv);
    args.AddOption(&mesh_file, "-mesh", "--mesh", "gmsh v2.2 mesh file (else a Cartesian square).");
    args.AddOption(&n, "-n", "--elems", "Elements per direction of the generated square.");
    args.AddOption(&order, "-p", "--order", "H1 order.");
    args.AddOption(&rs, "-rs", "--serial-ref-levels", "Uniform refinements before the partition.");
    args.AddOption(&rp, "-rp", "--par-ref-levels", "Uniform refinements after the partition.");
    args.AddOption(&alpha, "-a", "--alpha", "Diffusivity.");
    args.AddOption(&dt, "-dt", "--dt", "Time step.");
    args.AddOption(&t_final, "-T", "--t-final", "Final time.");
    args.AddOption(&opts, "-opts", "--petsc-options", "PETSc options file.");
    args.Parse();
    if (!args.Good()) {
        if (myid == 0) args.PrintUsage(cerr);
        return 1;
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

        H1_FECollection fec(order, pmesh->Dimension());
        ParFiniteElementSpace fespace(pmesh.get(), &fec);
        const HYPRE_BigInt global_true_dofs = fespace.GlobalTrueVSize();

        Array<int> ess_bdr(pmesh->bdr_attributes.Max());
        ess_bdr = 1;
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ExactCoefficient exact_coeff;
        ForcingCoefficient forcing_coeff(alpha);
        ConstantCoefficient alpha_dt_coeff(alpha * dt);

        ParBilinearForm mass_form(&fespace);
        mass_form.AddDomainIntegrator(new MassIntegrator());
        mass_form.Assemble();
        mass_form.Finalize();

        ParBilinearForm lhs_form(&fespace);
        lhs_form.AddDomainIntegrator(new MassIntegrator());
        lhs_form.AddDomainIntegrator(new DiffusionIntegrator(alpha_dt_coeff));
        lhs_form.Assemble();
        lhs_form.Finalize();

        ParGridFunction u(&fespace);
        ParGridFunction u_exact(&fespace);
        ParGridFunction u_error(&fespace);
        exact_coeff.SetTime(0.0);
        u.ProjectCoefficient(exact_coeff);
        u_exact.ProjectCoefficient(exact_coeff);
        u_error = 0.0;

        const int order_quad = max(2, 2 * order + 3);
        const IntegrationRule *irs[Geometry::NumGeom];
        for (int g = 0; g < Geometry::NumGeom; g++) irs[g] = &IntRules.Get(g, order_quad);

        const int nsteps = static_cast<int>(ceil(t_final / dt - 1.0e-12));
        Vector rhs_local(fespace.GetVSize());
        OperatorHandle Ah(Operator::Hypre_ParCSR);
        Vector X, B;
        long gmres_its = 0;
        double linf_err = 0.0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int step = 1; step <= nsteps; step++) {
            const double t = step * dt;
            mass_form.Mult(u, rhs_local);

            forcing_coeff.SetTime(t);
            ParLinearForm f_form(&fespace);
            f_form.AddDomainIntegrator(new DomainLFIntegrator(forcing_coeff));
            f_form.Assemble();
            rhs_local.Add(dt, f_form);

            exact_coeff.SetTime(t);
            u.ProjectBdrCoefficient(exact_coeff, ess_bdr);

            lhs_form.FormLinearSystem(ess_tdof_list, u, rhs_local, Ah, X, B);

            HypreParMatrix *A_hyp = Ah.As<HypreParMatrix>();
            MFEM_VERIFY(A_hyp != nullptr, "Expected HypreParMatrix.");
            PetscParMatrix A_petsc(A_hyp, Operator::PETSC_MATAIJ);
            PetscLinearSolver solver(A_petsc);
            solver.SetPrintLevel(0);
            solver.Mult(B, X);
            MFEM_VERIFY(solver.GetConverged(), "PETSc solver did not converge at step "
                                                   << step << ". Iterations=" << solver.GetNumIterations()
                                                   << ", residual=" << solver.GetFinalNorm());
            gmres_its += solver.GetNumIterations();

            lhs_form.RecoverFEMSolution(X, rhs_local, u);

            // Linf error, MPI-reduced (:375-383)
            u_exact.ProjectCoefficient(exact_coeff);
            subtract(u, u_exact, u_error);
            const double local_linf = u_error.Normlinf();
            MPI_Allreduce(&local_linf, &linf_err, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double t_end = nsteps * dt;
        exact_coeff.SetTime(t_end);
        const double final_l2 = u.ComputeL2Error(exact_coeff, irs);  // collective: every rank calls it
        if (myid == 0)
            std::printf("dofs %lld\nranks %d\nsteps %d\nfinal_l2 %.17g\nfinal_linf %.17g\ngmres_iterations %ld\n"
                        "seconds_per_step %.6g\n",
                        (long long)global_true_dofs, Mpi::WorldSize(), nsteps, final_l2, linf_err, gmres_its,
                        secs / std::max(nsteps, 1));
    } catch (const exception &e) {
        if (myid == 0) cerr << "Error: " << e.what() << endl;
        exit_code = 3;
    }

    MFEMFinalizePetsc();
    return exit_code;
}
